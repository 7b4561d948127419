// conv_halo.hip -- halo-tiled direct convolution for stride-1 R x S (<= 3 x 3) layers on CDNA4.
//
// The implicit-GEMM kernels of conv_fwd.hip stage an im2col B tile per (tap, channel chunk): a
// 3x3 conv moves every input element through the L2 -> LDS path 9 times. A 128 x 128 x 64 tile
// then does 64 FLOP per staged byte, and at the ~70 GB/s a CU draws from L2 the MFMA pipe runs
// at <= ~45 % (measured: the ResNet-50 3x3 layers at 500-650 TF/s, profiles/r4_*).
//
// Here a workgroup owns a SPATIAL output tile -- `th` whole output rows of one image -- times BC
// output channels. Per 64-channel
// input chunk the tile's input HALO ((th + R - 1) x (W + S - 1) pixels per image, zero padded)
// is staged ONCE into LDS by LDS-DMA, and all R*S taps read their B fragments from it at a
// uniform tap offset; only the weights [BC][64] of each (chunk, tap) step stream through a ring
// of D + 1 LDS buffers (D steps in flight). Staged bytes per FLOP drop ~3-5x (3x3 256@14, BC 128:
// 196 FLOP/B), which lifts the L2 bound above the MFMA rate.
//
// Semantics: y = conv(x, w) (+ residual) with the fused epilogue of conv_fwd.hip (next-BN
// statistics, or the fused BN-backward reduction of a data gradient) -- reference
// resnet_model_official.py:80-91 (conv2d_fixed_padding, SAME for stride 1), :153-175 (the
// bottleneck's 3x3). Stride-1 data gradients of 3x3 convs are the same op on the flipped,
// channel-transposed weights, so both directions run here.
//
// Layout: 8 waves = WAVES_P (pixel groups of MJ 16-pixel fragments) x WAVES_C (channel groups of
// MI 16-channel fragments); MFMA v_mfma_f32_16x16x32_bf16, A = weights (rows = output channels),
// B = halo pixels. LDS rows are 128 B (64 channels) with 16-byte slots XOR-swizzled (weights:
// (row >> 1) & 7 = glds_swz<64>, halo: halo_swz), both conflict-free for the ds_read_b128 fragment
// reads; the swizzle is applied on the per-lane SOURCE address of the lane-linear LDS-DMA.
#include "drn_common.h"
#include "drn_conv.h"
#include "drn_conv_epi.h"

namespace drn {

// Host-computed tile geometry (one launch). A tile is `th` output rows of one image; every row is
// cut into fpr 16-pixel fragments (the last one partly past the row end: garbage columns that are
// computed and never stored). A fragment therefore never wraps to the next row, so its 16 lanes
// read 16 CONSECUTIVE halo pixels at every tap, which halo_swz spreads over all 16-byte slots of
// a bank row (conflict-free ds_read_b128). Fragments wrapping an image row measured 39 % LDS bank
// conflicts, 16-pixel runs with the (row >> 1) & 7 swizzle 33 % (runs start unaligned).
struct HaloGeom {
  int32_t th;            // output rows per tile
  int32_t tpi;           // tiles per image = P / th
  int32_t fpr;           // 16-pixel fragments per output row = ceil(Q / 16)
  int32_t hh, hw;        // halo rows (th + R - 1), halo columns (Q + S - 1)
  int32_t hpx;           // halo pixels of a tile = hh * hw
  int32_t ntp;           // pixel tiles = N * tpi
};

// staged epilogue row -> output pixel (>= M for garbage columns / fragments past the tile)
struct EpiRowHalo {
  int fpr, Q, th, M;
  __device__ __forceinline__ int operator()(int m0, int row) const {
    const int f = row >> 4;
    const int r = f / fpr;
    const int c = (f - r * fpr) * 16 + (row & 15);
    return (r < th && c < Q) ? m0 + r * Q + c : M;
  }
};

// 16-byte slot swizzle of the halo image: logical chunk c of halo pixel hp sits in slot
// c ^ (hp & 6). Unlike the (hp >> 1) & 7 swizzle of the implicit-GEMM tiles (conflict-free only
// for 16-aligned row groups), it keeps ds_read_b128 conflict-free for a fragment's 16 consecutive
// halo pixels at ANY start (a tap shifts the run by dr * hw + ds): exhaustive check over the four
// gfx950 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... and both k halves.
__device__ __forceinline__ int halo_swz(int hp) { return hp & 6; }

// s_waitcnt vmcnt(n) for a run-time n (0..30), off the steady-state path
__device__ __noinline__ void wait_vmcnt_rt(int n) {
  switch (n) {
#define DRN_W(k) \
  case k:        \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
    DRN_W(0) DRN_W(1) DRN_W(2) DRN_W(3) DRN_W(4) DRN_W(5) DRN_W(6) DRN_W(7) DRN_W(8) DRN_W(9) DRN_W(10)
    DRN_W(11) DRN_W(12) DRN_W(13) DRN_W(14) DRN_W(15) DRN_W(16) DRN_W(17) DRN_W(18) DRN_W(19) DRN_W(20)
    DRN_W(21) DRN_W(22) DRN_W(23) DRN_W(24) DRN_W(25) DRN_W(26) DRN_W(27) DRN_W(28) DRN_W(29) DRN_W(30)
#undef DRN_W
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// MJ pixel fragments per wave; HPW = max halo pieces (8 pixels x 128 B each) per wave
template <int WAVES_P, int MJ, int WAVES_C, int MI, int D, int HPW, bool PRO>
__global__ __launch_bounds__(512) void conv_halo_kernel(DrnConvFwdArgs a, HaloGeom g, const void* __restrict__ zero) {
  constexpr int NW = 8, NT = 512;
  static_assert(WAVES_P * WAVES_C == NW, "8 waves");
  constexpr int BP = WAVES_P * MJ * 16;   // computed pixel columns (th * fpr * 16 <= BP)
  constexpr int BC = WAVES_C * MI * 16;   // output channels per tile
  constexpr int WP = MJ * 16, WC = MI * 16;
  constexpr int NWB = D + 1;              // weight ring buffers
  constexpr int GW = BC / 64;             // weight glds pieces per wave per step (BC rows x 128 B / 8 waves)
  constexpr int STEADY = (D - 1) * GW;    // loads left in flight at a steady-state step
  static_assert(GW >= 1 && GW * 64 == BC, "BC multiple of 64");
  static_assert(HPW % 4 == 0, "halo pieces per wave: batches of 4");
  static_assert(D >= 2 && STEADY < 31, "pipeline depth");
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.C, K = a.K, S = a.S;
  const int RS = a.R * S;
  const int nchunk = C >> 6;
  const int T = nchunk * RS;              // steps (chunk-major, tap-minor)
  const int M = a.N * a.P * a.Q;
  const int ntc = K / BC;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tcol = bid % ntc, tpix = bid / ntc;
  const int c0 = tcol * BC;
  const int n0 = tpix / g.tpi;
  const int p0 = (tpix - n0 * g.tpi) * g.th;
  const int m0 = (n0 * a.P + p0) * a.Q;

  // LDS: [halo buffer 0][halo buffer 1 (nchunk > 1)][NWB weight buffers][PRO: scale C, shift C];
  // a halo buffer holds the tile's halo plus 2 spare KB read by the garbage columns of the last
  // fragment of a row
  const int npieces = (g.hpx + 7) >> 3;
  const int hbytes = (npieces + 2) << 10;
  char* const wbuf0 = smem + (nchunk > 1 ? 2 : 1) * hbytes;
  constexpr int WBYTES = BC * 128;
  float* const ssl = reinterpret_cast<float*>(wbuf0 + NWB * WBYTES);

  // ---- halo loader: per-lane source offsets of this wave's pieces (element offset at chunk 0,
  // -1 = outside the image: the zero page) ----
  const int my_pieces = npieces > wave ? (npieces - wave + NW - 1) / NW : 0;  // wave-uniform
  int hoff[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int hp = (i * NW + wave) * 8 + (lane >> 3);
    int off = -1;
    if (i < my_pieces && hp < g.hpx) {
      const int ar = hp / g.hw;
      const int bc = hp - ar * g.hw;
      const int h = p0 - a.pad_h + ar;
      const int w = bc - a.pad_w;
      if ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
        off = ((n0 * a.H + h) * a.W + w) * C + (((lane & 7) ^ halo_swz(hp)) << 3);
    }
    hoff[i] = off;
  }
  const bf16_t* __restrict__ xg = reinterpret_cast<const bf16_t*>(a.x);
  auto issue_halo = [&](int chunk, char* hb) {
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      if (i < my_pieces) {
        const void* src = hoff[i] >= 0 ? (const void*)(xg + hoff[i] + (chunk << 6)) : zero;
        glds16(src, hb + ((i * NW + wave) << 10));
      }
    }
  };
  // ---- weight loader: rows c0 + row of w[K][R][S][C], 64 channels of one (tap, chunk) ----
  const bf16_t* __restrict__ wrow;
  {
    const int row = wave * 8 + (lane >> 3);  // + i * 64 rows for piece i
    wrow = reinterpret_cast<const bf16_t*>(a.w) + (size_t)(c0 + row) * (RS * C) + (((lane & 7) ^ glds_swz<64>(row)) << 3);
  }
  const size_t wpiece = (size_t)64 * RS * C;  // 64 rows further (the swizzle bits repeat every 16 rows)
  auto issue_w = [&](int koff, int slot) {   // koff = tap * C + chunk * 64
    char* wb = wbuf0 + slot * WBYTES;
#pragma unroll
    for (int i = 0; i < GW; ++i) glds16(wrow + i * wpiece + koff, wb + ((i * NW + wave) << 10));
  };

  // ---- fragment addressing ----
  const int wp = wave % WAVES_P, wc = wave / WAVES_P;
  const int fr = lane & 15, fk = lane >> 4;
  // B: fragment f = (row f / fpr, columns (f % fpr) * 16 ..) -> halo pixel of tap (0, 0)
  int hb0[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int f = wp * MJ + j;
    const int r = f / g.fpr;
    const int c = (f - r * g.fpr) * 16 + fr;
    hb0[j] = (r < g.th ? r : 0) * g.hw + c;  // (fragments past the tile read row 0: garbage, not stored)
  }
  uint32_t aoff[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int row = wc * WC + i * 16 + fr;  // 16-aligned groups: the swizzle bits are fr's
    aoff[i] = (uint32_t)(row * 128 + ((fk ^ glds_swz<64>(fr)) << 4));
  }

  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: halo of chunk 0, weights of steps 0 .. D-1 (tap-minor k offsets) ----
  issue_halo(0, smem);
  // PRO: the input is the raw pre-BN tensor; relu(x * scale + shift) is applied to the halo ONCE
  // per chunk in LDS (each lane rewrites the 16-byte pieces its own LDS-DMAs landed, before the
  // chunk's first barrier; zero-padding pieces stay zero) -- 1/(R*S) of the per-tap rewrite an
  // im2col tile needs. scale / shift of every channel are staged in LDS behind the buffers (or
  // finalized there from the BN statistics: consumer-side finalize, DrnBnFin).
  if constexpr (PRO) {
    if (a.in_fin.stats != nullptr) {
      const bool pub = a.in_fin.publish && blockIdx.x == 0;
      for (int c = tid; c < C; c += NT) drn_bn_fin_fwd(a.in_fin, c, pub, ssl[c], ssl[C + c]);
    } else {
      for (int c = tid; c < C; c += NT) {
        ssl[c] = a.in_scale[c];
        ssl[C + c] = a.in_shift[c];
      }
    }
    __syncthreads();
  }
  // the lane's logical chunk inside a halo piece: (lane & 7) ^ halo_swz(hp) with hp & 6 = the
  // bits 1-2 of lane >> 3 for every piece (pieces are 8-pixel aligned)
  const int plc = (lane & 7) ^ halo_swz(lane >> 3);
  auto transform_halo = [&](int chunk, char* hb) {
    const uint32_t sp = lds_addr(ssl + (chunk << 6) + plc * 8);
    u32x4_t q[4];
    q[0] = lds_read16(sp);
    q[1] = lds_read16(sp + 16);
    q[2] = lds_read16(sp + 4 * C);
    q[3] = lds_read16(sp + 4 * C + 16);
    lds_wait_all<4>(q);
    f32x2_t sc2[4], sh2[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      sc2[2 * k] = f32x2_t{__uint_as_float(q[k][0]), __uint_as_float(q[k][1])};
      sc2[2 * k + 1] = f32x2_t{__uint_as_float(q[k][2]), __uint_as_float(q[k][3])};
      sh2[2 * k] = f32x2_t{__uint_as_float(q[2 + k][0]), __uint_as_float(q[2 + k][1])};
      sh2[2 * k + 1] = f32x2_t{__uint_as_float(q[2 + k][2]), __uint_as_float(q[2 + k][3])};
    }
    // in batches of 4 pieces (registers: the accumulators and prefetched fragments are live)
#pragma unroll
    for (int i0 = 0; i0 < HPW; i0 += 4) {
      u32x4_t v[4];
      uint32_t pa[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        pa[k] = lds_addr(hb + (((i0 + k) * NW + wave) << 10) + lane * 16);
        if (i0 + k < my_pieces) v[k] = lds_read16(pa[k]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (i0 + k < my_pieces) {
          u32x4_t o = bn_relu_piece<true>(v[k], sc2, sh2);
          const unsigned m = hoff[i0 + k] >= 0 ? 0xffffffffu : 0u;  // zero-page pieces stay zero
          o.x &= m;
          o.y &= m;
          o.z &= m;
          o.w &= m;
          lds_write16(pa[k], o);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  int wtap = 0, wchunk = 0, wslot = 0, wstep = 0;
  auto issue_next_w = [&]() {
    issue_w(wtap * C + (wchunk << 6), wslot);
    if (++wtap == RS) {
      wtap = 0;
      ++wchunk;
    }
    wslot = wslot + 1 == NWB ? 0 : wslot + 1;
    ++wstep;
  };
#pragma unroll
  for (int s = 0; s < D; ++s)
    if (wstep < T) issue_next_w();

  const uint32_t lds0 = lds_addr(smem);
  const uint32_t wlds0 = lds0 + (uint32_t)(wbuf0 - smem);
  int tap = 0, chunk = 0, dr = 0, ds = 0, cslot = 0;
  u32x4_t bv[2][MJ];  // this step's B fragments (k halves 0, 1)
  for (int s = 0; s < T; ++s) {
    // loads allowed to stay in flight: the weights of steps s+1 .. s+D-1, plus the halo batch of
    // the next chunk when it was issued after W(s) (at the chunk's first step, < D steps ago;
    // R*S >= D: at most one batch)
    const int ahead = T - 1 - s < D - 1 ? T - 1 - s : D - 1;
    const int allowed = ahead * GW + ((chunk + 1 < nchunk && tap >= 1 && tap <= D - 1) ? my_pieces : 0);
    if (allowed == STEADY) wait_vmcnt<STEADY>();
    else wait_vmcnt_rt(allowed);
    if constexpr (PRO) {
      if (tap == 0) transform_halo(chunk, smem + (chunk & 1) * hbytes);  // this chunk's halo landed
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (tap == 0 && chunk + 1 < nchunk) issue_halo(chunk + 1, smem + ((chunk + 1) & 1) * hbytes);
    if (wstep < T) issue_next_w();
    const uint32_t hbase = lds0 + (uint32_t)((chunk & 1) * hbytes);
    const uint32_t wbase = wlds0 + (uint32_t)(cslot * WBYTES);
    // B fragments of this step: prefetched during the previous step when it was in the same
    // chunk (the halo buffer is stable for a whole chunk), else read now
    if (tap == 0) {
      const int toff = dr * g.hw + ds;
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int hp = hb0[j] + toff;
        const uint32_t ad = hbase + (uint32_t)(hp << 7) + (uint32_t)((fk ^ halo_swz(hp)) << 4);
        bv[0][j] = lds_read16(ad);
        bv[1][j] = lds_read16(ad ^ 64u);
      }
    }
    // A fragments (k halves 0 and 1: slot ^ 4 = LDS address ^ 64)
    u32x4_t av[2][MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      av[0][i] = lds_read16(wbase + aoff[i]);
      av[1][i] = lds_read16((wbase + aoff[i]) ^ 64u);
    }
    // next step's B fragments, in flight during this step's MFMAs
    const bool pre = tap + 1 < RS;
    u32x4_t bn[2][MJ];
    if (pre) {
      const int ds1 = ds + 1 == S ? 0 : ds + 1, dr1 = ds + 1 == S ? dr + 1 : dr;
      const int toff = dr1 * g.hw + ds1;
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int hp = hb0[j] + toff;
        const uint32_t ad = hbase + (uint32_t)(hp << 7) + (uint32_t)((fk ^ halo_swz(hp)) << 4);
        bn[0][j] = lds_read16(ad);
        bn[1][j] = lds_read16(ad ^ 64u);
      }
      static_assert(2 * MJ <= 15, "lgkmcnt range");
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * MJ) : "memory");  // this step's A and B landed
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av[kh][i]),
                                                              __builtin_bit_cast(bf16x8_t, bv[kh][j]), acc[i][j], 0, 0,
                                                              0);
    if (pre) {
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        bv[0][j] = bn[0][j];
        bv[1][j] = bn[1][j];
      }
    }
    // advance the compute step (incremental: no scalar divisions in the loop)
    cslot = cslot + 1 == NWB ? 0 : cslot + 1;
    if (++ds == S) {
      ds = 0;
      ++dr;
    }
    if (++tap == RS) {
      tap = dr = ds = 0;
      ++chunk;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every fragment read done before the epilogue reuses the LDS
  const EpiRowHalo rmap{g.fpr, a.Q, g.th, M};
  constexpr int NH = (BP * BC * 4 > 160 * 1024) ? 2 : 1;
  if constexpr (NH == 1) {
    EpiPre<BP, BC, NT, false> epre;  // (unused: lazy per-row offsets through the row map)
    conv_epilogue_pass<BP, BC, WP, MI, MJ, NT, false, true, EpiRowHalo>(a, smem, acc, true, wp, wc * WC, m0, c0, M,
                                                                        epre, rmap);
  } else {
    conv_epilogue_sliced<BP, BC, WP, WC, MI, MJ, NT, NH, EpiRowHalo>(a, smem, acc, wp, wc, m0, c0, M, rmap);
  }
}

// configurations: {WAVES_P, MJ, WAVES_C, MI, D}
//   0: 224 px x 128 ch (28x28 / 14x14 / 7x7 stages), 3 steps in flight
//   1: 256 px x 64 ch (56x56, 64 channels), 3 in flight
//   2: 448 px x 64 ch (56x56, 8 rows per tile)
//   3: 256 px x 128 ch, 4 x 4 fragments per wave (32 FLOP per LDS byte), 2 in flight
//   4: 128 px x 128 ch (7x7: 2 images per tile)
//   5: 256 px x 64 ch, every wave all 64 channels of 32 pixels
#define DRN_HALO_CONFIGS(X) \
  X(0, 2, 7, 4, 2, 3)       \
  X(1, 4, 4, 2, 2, 3)       \
  X(2, 4, 7, 2, 2, 3)       \
  X(3, 4, 4, 2, 4, 2)       \
  X(4, 2, 4, 4, 2, 3)       \
  X(5, 8, 2, 1, 4, 3)
#define DRN_HALO_NCFG 6
#define DRN_HALO_HPW 8

// tile geometry for a computed pixel width BP: the most output rows th (th | P) whose fragments
// (fpr per row) fit BP; 0 if not even one row fits
static int halo_geom(const DrnConvFwdArgs* a, int BP, HaloGeom* g) {
  const int P = a->P, Q = a->Q;
  g->fpr = (Q + 15) / 16;
  g->th = 0;
  for (int th = P; th >= 1; --th)
    if (P % th == 0 && th * g->fpr * 16 <= BP) {
      g->th = th;
      break;
    }
  if (g->th == 0) return 0;
  g->tpi = P / g->th;
  g->hh = g->th + a->R - 1;
  g->hw = Q + a->S - 1;
  g->hpx = g->hh * g->hw;
  g->ntp = a->N * g->tpi;
  return 1;
}

template <int WAVES_P, int MJ, int WAVES_C, int MI, int D, bool PRO>
static int launch_halo(const DrnConvFwdArgs* a, const void* zero, hipStream_t s) {
  constexpr int BP = WAVES_P * MJ * 16, BC = WAVES_C * MI * 16;
  if (a->K % BC || a->R * a->S < D) return (int)hipErrorInvalidValue;
  HaloGeom g;
  if (!halo_geom(a, BP, &g)) return (int)hipErrorInvalidValue;
  const int npieces = (g.hpx + 7) / 8;
  if ((npieces + 7) / 8 > DRN_HALO_HPW) return (int)hipErrorInvalidValue;
  // the spare halo KB must cover the garbage columns' reach past the halo (fpr*16 - Q + S - 1 px)
  if (g.fpr * 16 - a->Q + a->S - 1 > 16) return (int)hipErrorInvalidValue;
  const int nchunk = a->C / 64;
  const int hbytes = (npieces + 2) * 1024;
  const int lds_main = (nchunk > 1 ? 2 : 1) * hbytes + (D + 1) * BC * 128 + (PRO ? 8 * a->C : 0);
  constexpr int NH = (BP * BC * 4 > 160 * 1024) ? 2 : 1;
  const int lds_epi = BP * BC * 4 / NH;
  const int lds = lds_main > lds_epi ? lds_main : lds_epi;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  // the runtime vmcnt switch covers counts up to 30
  if ((D - 1) * (BC / 64) + (npieces + 7) / 8 > 30) return (int)hipErrorInvalidValue;
  if (PRO && a->in_fin.stats != nullptr &&
      (a->in_fin.C != a->C || a->in_fin.G < 1 || a->in_fin.G > DRN_BN_FIN_GMAX))
    return (int)hipErrorInvalidValue;
  auto kern = conv_halo_kernel<WAVES_P, MJ, WAVES_C, MI, D, DRN_HALO_HPW, PRO>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  const int grid = g.ntp * (a->K / BC);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, s, *a, g, zero);
  return (int)hipGetLastError();
}

}  // namespace drn

// Whether the halo kernel family supports this convolution (stride 1, R, S <= 3 with SAME
// padding, 64-channel chunks, identity output map; a fused BN-apply + ReLU input prologue is
// supported, the BN-backward input transform is not).
DRN_API int drn_conv_halo_ok(const DrnConvFwdArgs* a) {
  return a->stride == 1 && a->dil == 1 && a->R <= 3 && a->S <= 3 && a->R >= 1 && a->S >= 1 && a->C % 64 == 0 &&
         a->C <= 4096 && a->K % 64 == 0 && (a->in_scale == nullptr || a->relu_in != 0) && a->bnb_x == nullptr &&
         a->out_stride == 0 && a->ksplit <= 1 &&
         a->sk_blocks == 0 && a->fin_cnt == nullptr && a->P == a->H && a->Q == a->W && a->pad_h >= 0 &&
         a->pad_w >= 0 && a->pad_h < a->R && a->pad_w < a->S;
}

DRN_API int drn_conv_halo_num_cfgs() { return DRN_HALO_NCFG; }

DRN_API int drn_conv_halo(int cfg, const DrnConvFwdArgs* a, const void* zero, hipStream_t s) {
  if (!drn_conv_halo_ok(a) || zero == nullptr) return (int)hipErrorInvalidValue;
  switch (cfg) {
#define DRN_X(id, wp, mj, wc, mi, d)                                                      \
  case id:                                                                                \
    return a->in_scale != nullptr ? drn::launch_halo<wp, mj, wc, mi, d, true>(a, zero, s) \
                                  : drn::launch_halo<wp, mj, wc, mi, d, false>(a, zero, s);
    DRN_HALO_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return (int)hipErrorInvalidValue;
  }
}
