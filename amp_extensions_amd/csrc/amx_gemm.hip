// fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32, exact f32 fma chains) with
// fused epilogues for the hot path of the learned-dynamics rollout:
//   * bias + ReLU written into a column slice of the dense-concat activation row
//     (BasicMLP hidden layers, milo/milo/dynamics.py:427-430),
//   * bias + output un-normalisation (milo/milo/dynamics.py:231-232),
//   * bias + cos * sqrt(2/F) random Fourier features with fp64 column sums
//     (RBFLinearCost.get_rep / fit_cost, milo/milo/linear_cost.py:64-94).
//
// C[r][n] = sum_k A[r][k] * W[n][k]: both operands are K-contiguous ("NT"), which is the
// torch nn.Linear weight layout, so weights are used as stored.
//
// Tile family Tile<WM, WN, TM, TN>: WM x WN waves, each owning TM x TN MFMA 32x32 tiles, so
// the workgroup tile is (32*WM*TM) x (32*WN*TN) with BK = 32.  Operands are register-staged
// through LDS (double buffer, one barrier per K-tile, the next tile's global loads issued
// before the MFMA block).  Lane l of an MFMA supplies k-slot h = l>>5; slot h of MFMA step s
// is mapped to k = 16h + s, so each lane reads 16 consecutive floats of its row with 4
// ds_read_b128 (the same permutation on A and W keeps the contraction exact).  LDS rows are
// padded to 36 floats: rows 16 apart land on distinct 16-byte bank slots, so the 16-lane
// groups of ds_read_b128 are conflict-free.
#include "amx_common.h"
#include "amx_h3.h"

#include <type_traits>

// H3_TRACE (diagnostic builds, tools/h3_trace.py): thread 0 of every workgroup of an f16x3
// launch stamps the device realtime clock (100 MHz) at the phases of its tile -- 0 entry, 1 row
// exponents read, 2 K loop entered, 3 K loop done, 4 epilogue issued, 5 its stores drained --
// into h3_trace_buf[K / 512 % 5][block] (the forward's five layers: K 256 .. 2304)
#ifndef H3_TRACE
#define H3_TRACE 0
#endif
#if H3_TRACE
__device__ unsigned long long h3_trace_buf[5][1024][8];
#define H3_STAMP(a, ph)                                                                        \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 1024)                                                 \
      h3_trace_buf[((a).K / 512) % 5][blockIdx.x][ph] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
extern "C" int amx_h3_trace_read(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(h3_trace_buf), sizeof(h3_trace_buf)) == hipSuccess ? 0 : -1;
}
#else
#define H3_STAMP(a, ph) \
  do {                  \
  } while (0)
#endif

namespace {


constexpr int BK = 32;
constexpr int LDS_LD = BK + 4;  // floats per LDS row


template <int WM_, int WN_, int TM_, int TN_>
struct Tile {
  static constexpr int WM = WM_, WN = WN_, TM = TM_, TN = TN_;
  static constexpr int OCC = 2;                             // __launch_bounds__ waves-per-SIMD target
  static constexpr int NT = WM * WN * 64;
  static constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  static constexpr int STAGE = (BM + BN) * LDS_LD;          // floats of one stage (A + W)
  static constexpr size_t LDS = 2 * STAGE * sizeof(float);  // double-buffered, 1 barrier / K-tile
  static constexpr int ROW_STEP = NT / 8;                   // staging rows covered per pass
  static constexpr int VA = BM / ROW_STEP, VW = BN / ROW_STEP;
  static_assert(BM % ROW_STEP == 0 && BN % ROW_STEP == 0, "staging map");
  static_assert(LDS <= 160 * 1024, "LDS");
};


// LDS of the RFF epilogue: the staged BM x (BN + 4) f32 tile
constexpr size_t rff_epi_lds(int bm, int bn) { return (size_t)bm * (bn + 4) * 4; }
// rows of the M16 RFF epilogue's staging pass: the whole tile when its [BM][BN + 4] floats fit
// 80 KB, else the largest multiple of 32 rows that does (the 160 x 256 tile: 64 rows)
constexpr int rff_m16_rows(int bm, int bn) {
  return rff_epi_lds(bm, bn) <= 80 * 1024 ? bm : (int)((80 * 1024) / ((size_t)(bn + 4) * 4 * 32)) * 32;
}

// ---- epilogue (shared by the f32 and the bf16x6 main loops: the 32x32 C/D register map
// is dtype-independent on gfx950) ---------------------------------------------------------
// Row validity of `n` <= 64 consecutive rows from `row0` (row < n_valid and row_mask[row] != 0)
// as a wave-uniform bit mask: lane l tests row row0 + l, a ballot gathers the bits.  The RFF
// epilogues test bit i per row from this mask instead of reading a per-row flag from LDS, so
// no LDS address is read by every lane of a wave at once.
__device__ __forceinline__ uint64_t row_valid_mask(const GemmArgs& a, int row0, int n) {
  const int l = threadIdx.x & 63, row = row0 + l;
  const bool v = l < n && row < a.n_valid && (a.row_mask == nullptr || a.row_mask[row] != 0);
  return __ballot(v);
}

// H3_EXP (diagnostic builds, bits): 1 = the split schedule's K-loop global loads left out (stale
// tiles), 2 = the A limb split left out (raw bits published)
#ifndef H3_EXP
#define H3_EXP 0
#endif
// H3_ORDERED_LOADS (A/B builds: 0 = the scheduler's order): the f16x3 K loop's prologue issues
// its staging loads in the loop's piece order (h3_tile's `load`)
#ifndef H3_ORDERED_LOADS
#define H3_ORDERED_LOADS 1
#endif
// H3_AFFINE (A/B builds: 0 = per-chunk offset registers): the 16x16x32 tiles' staging chunks j
// sit NT / CPR rows apart, so a chunk's global offset is chunk 0's plus a wave-uniform step
// (the buffer load's SGPR offset) and its LDS offset chunk 0's plus an immediate -- one
// address register per operand instead of one per chunk
#ifndef H3_AFFINE
#define H3_AFFINE 1
#endif
// H3_W4 (A/B builds): the hidden layers' 256 x 256 tile on 4 waves of 128 x 128 (one wave per
// SIMD, 256 accumulator registers each) instead of 8 waves of 128 x 64
#ifndef H3_W4
#define H3_W4 0
#endif
// OUT80 (A/B builds): 1 = the 80 x 224 output tile where it makes exactly one tile per CU
#ifndef OUT80
#define OUT80 1
#endif
// RFF_OCC3 (A/B builds): 1 = the RFF pass on 128 x 128 tiles at three workgroups per CU (H128rff3)
// when its tiles exceed one round at two per CU
#ifndef RFF_OCC3
#define RFF_OCC3 1
#endif
// RFF_EXP (diagnostic builds, tools/src_variant.sh): 1 = no cos, 2 = no phi store
#ifndef RFF_EXP
#define RFF_EXP 0
#endif
// cos for the RFF epilogues.  RFF_HWCOS 1: z reduced to r in [-pi, pi] by a Cody-Waite step
// (k = rint(z / 2 pi), 2 pi in three parts, fma), then the hardware v_cos_f32 on r / 2 pi; max
// |error| 3.5e-7 against cos((double) z) over |z| <= 4096 (tools/cos_accuracy.hip,
// profiles/r04o_cos_accuracy.txt: OCML cosf 7e-8), far below the fp32 rounding of the
// argument itself (|z| 2^-24: 6e-6 at the MILO features' |z| ~ 1e2); |z| >= 2^16 takes cosf.
// RFF_HWCOS 0: OCML cosf (rounds 1-3).
#ifndef RFF_HWCOS
#define RFF_HWCOS 1
#endif
__device__ __forceinline__ float rff_cos(float z) {
#if RFF_HWCOS
  if (__builtin_expect(__builtin_fabsf(z) >= 65536.0f, 0)) return cosf(z);
  const float k = __builtin_rintf(z * 0.15915494309189535f);
  float r = __builtin_fmaf(-k, 6.28318548202514648f, z);
  r = __builtin_fmaf(-k, -1.7484555314695172e-7f, r);
  r = __builtin_fmaf(-k, -2.3889859e-15f, r);
  return __builtin_amdgcn_cosf(r * 0.15915494309189535f);
#else
  return cosf(z);
#endif
}

template <int EPI, class TL>
__device__ __forceinline__ void epilogue(const GemmArgs& a, f32x16 (&acc)[TL::TM][TL::TN], int g, int tm, int tn) {
  constexpr int BM = TL::BM, BN = TL::BN, TM = TL::TM, TN = TL::TN;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int li = lane & 31, lh = lane >> 5;
  // C/D map of 32x32 f32 MFMA: column = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
  const int row0 = tm * BM + wm * TM * 32;
  const int col0 = tn * BN + wn * TN * 32;

  if constexpr (EPI == EPI_BIAS_ACT) {
    const float* bias = a.bias + (long long)g * a.strideBias;
    float* Cg = a.C + (long long)g * a.strideC;
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int col = col0 + n * 32 + li;
      const float bv = bias[col];
#pragma unroll
      for (int m = 0; m < TM; ++m) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = row0 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          float v = acc[m][n][e] + bv;
          if (a.act == AMX_ACT_RELU) v = (v < 0.f) ? 0.f : v;  // keeps NaN, as torch.relu
          Cg[(long long)row * a.ldc + a.col_off + col] = v;
        }
      }
    }
  } else if constexpr (EPI == EPI_UNNORM) {
    const float* bias = a.bias + (long long)g * a.strideBias;
    float* Cg = a.C + (long long)g * a.strideC;
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int col = col0 + n * 32 + li;
      if (col < a.n_valid) {
        const float bv = bias[col];
        const float sc = a.scale[col], sh = a.shift[col];
#pragma unroll
        for (int m = 0; m < TM; ++m) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = row0 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
            const float y = acc[m][n][e] + bv;
            const float prod = y * sc;    // two roundings, as torch's (y*scale)+mean
            Cg[(long long)row * a.ldc + col] = prod + sh;
          }
        }
      }
    }
  } else if constexpr (TL::OCC >= 3) {  // EPI_RFF, 128 x 128 tiles at three workgroups per CU
    // The staged epilogue below in two passes of the 64 rows of one wave row (wm = pass), so
    // the staging takes 64 x 132 floats (33.8 KB) and the tile's 41.5 KB of BK-16 stage
    // buffers set the LDS: three workgroups per CU.  Thread (c, part): column c, rows
    // 32 part .. + 31 of each pass: one fp64 partial per 32-row group (AMX_RFF_PART_ROWS),
    // summed in row order.
    static_assert(BM == 128 && BN == 128 && TL::NT == 256 && TL::WM == 2 && TM * 32 == 64, "RFF half epilogue");
    constexpr int CLD = BN + 4;
    float* Cs = smem;  // [64][CLD]
    const int c = t & (BN - 1), part = t / BN;
    const int col = tn * BN + c;
    const float bv = a.bias[col];
    float* Cg = a.C;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (wm == pass) {
#pragma unroll
        for (int n = 0; n < TN; ++n)
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int r = m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
              Cs[r * CLD + wn * TN * 32 + n * 32 + li] = acc[m][n][e];
            }
      }
      const int row0 = tm * BM + pass * 64 + part * 32;
      const uint64_t vmask = row_valid_mask(a, row0, 32);
      __syncthreads();
      double csum = 0.0;
#pragma unroll 8
      for (int i = 0; i < 32; ++i) {
        const int r = part * 32 + i;
        const float z = Cs[r * CLD + c] + bv;       // nn.Linear: x W^T + b
        const float phi = rff_cos(z) * a.rff_scale;  // torch.cos(.) * np.sqrt(2/F)
        Cg[(long long)(row0 + i) * a.ldc + col] = phi;
        csum += ((vmask >> i) & 1u) ? (double)phi : 0.0;
      }
      a.col_partials[(long long)(row0 / AMX_RFF_PART_ROWS) * a.N + col] = csum;
      __syncthreads();
    }
  } else {  // EPI_RFF (128 x 128 or 128 x 64 tiles of 256 threads)
    static_assert(BM == 128 && (BN == 128 || BN == 64) && TL::NT == 256, "RFF epilogue tiles");
    // Stage the raw BM x BN tile through LDS, then one column per thread over BM / PARTS rows:
    // coalesced phi rows, the cos of 8 rows in flight (unroll 8: 94-101 vs 102-112 us for the
    // 40 960-row pass, same bits; full unrolling is slower), and one fp64 partial per 32-row
    // group (AMX_RFF_PART_ROWS) of the valid rows in row order (2 groups per thread at BN 128,
    // 1 at BN 64).
    constexpr int CLD = BN + 4, PARTS = 256 / BN, PR = BM / PARTS;
    static_assert(PR % AMX_RFF_PART_ROWS == 0, "whole partial groups per thread");
    float* Cs = smem;  // [BM][CLD] (rff_epi_lds), reuses the stage buffers (last barrier passed)
#pragma unroll
    for (int n = 0; n < TN; ++n)
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = wm * TM * 32 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          Cs[r * CLD + wn * TN * 32 + n * 32 + li] = acc[m][n][e];
        }
    const int c = t & (BN - 1), part = t / BN;  // part is wave-uniform (BN >= 64)
    // the validity (n_valid, row_mask) of the wave's PR <= 64 rows as one wave-uniform bit mask:
    // lane l loads row part*PR + l (lane-distinct, coalesced), a ballot forms the mask
    const uint64_t vmask = row_valid_mask(a, tm * BM + part * PR, PR);
    __syncthreads();
    const int col = tn * BN + c;
    const float bv = a.bias[col];
    float* Cg = a.C;
#pragma unroll
    for (int q = 0; q < PR / AMX_RFF_PART_ROWS; ++q) {
      double csum = 0.0;
#pragma unroll 8
      for (int i = q * AMX_RFF_PART_ROWS; i < (q + 1) * AMX_RFF_PART_ROWS; ++i) {
        const int r = part * PR + i;
        const int row = tm * BM + r;
        const float z = Cs[r * CLD + c] + bv;       // nn.Linear: x W^T + b
#if RFF_EXP == 1
        const float phi = z * a.rff_scale;
#else
        const float phi = rff_cos(z) * a.rff_scale;  // torch.cos(.) * np.sqrt(2/F)
#endif
#if RFF_EXP != 2
        Cg[(long long)row * a.ldc + col] = phi;
#endif
        csum += ((vmask >> i) & 1u) ? (double)phi : 0.0;
      }
      a.col_partials[(long long)((tm * BM + part * PR) / AMX_RFF_PART_ROWS + q) * a.N + col] = csum;
    }
  }
}

// One output tile (linear id `orig`, see map_tile) of the grouped GEMM.
template <int EPI, class TL>
__device__ __forceinline__ void gemm_tile(const GemmArgs& a, int orig) {
  constexpr int BM = TL::BM, BN = TL::BN, TM = TL::TM, TN = TL::TN, VA = TL::VA, VW = TL::VW;
  constexpr int STAGE = TL::STAGE, RS = TL::ROW_STEP;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int g, tm, tn;
  map_tile(a, orig, g, tm, tn);
  const float* __restrict__ Ag = a.A + (long long)g * a.strideA + (long long)tm * BM * a.lda;
  const float* __restrict__ Wg = a.W + (long long)g * a.strideW + (long long)tn * BN * a.ldw;

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int li = lane & 31, lh = lane >> 5;

  // staging map: float4 q = t + NT*j -> row (t>>3) + RS*j, column 4*(t&7).  The stage
  // registers stay in registers: the loops below are fully unrolled with constant indices
  // and no lambda captures them (a captured array went to scratch in an earlier version).
  const int st_r = t >> 3, st_c = (t & 7) * 4;
  const float* a_src = Ag + (long long)st_r * a.lda + st_c;
  const float* w_src = Wg + (long long)st_r * a.ldw + st_c;
  const long long a_step = (long long)RS * a.lda, w_step = (long long)RS * a.ldw;
  float* const a_dst0 = smem + st_r * LDS_LD + st_c;
  float* const w_dst0 = smem + BM * LDS_LD + st_r * LDS_LD + st_c;

  f32x4 ra[VA], rw[VW];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = a.K / BK;
#pragma unroll
  for (int j = 0; j < VA; ++j) ra[j] = *reinterpret_cast<const f32x4*>(a_src + j * a_step);
#pragma unroll
  for (int j = 0; j < VW; ++j) rw[j] = *reinterpret_cast<const f32x4*>(w_src + j * w_step);
#pragma unroll
  for (int j = 0; j < VA; ++j) *reinterpret_cast<f32x4*>(a_dst0 + j * RS * LDS_LD) = ra[j];
#pragma unroll
  for (int j = 0; j < VW; ++j) *reinterpret_cast<f32x4*>(w_dst0 + j * RS * LDS_LD) = rw[j];
  __syncthreads();

  const int a_off = (wm * TM * 32 + li) * LDS_LD + lh * 16;
  const int w_off = BM * LDS_LD + (wn * TN * 32 + li) * LDS_LD + lh * 16;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // prefetch the next K-tile (the last iteration re-reads its own tile: branch-free loop)
    const int kn = (kt + 1 < nk ? kt + 1 : kt) * BK;
#pragma unroll
    for (int j = 0; j < VA; ++j) ra[j] = *reinterpret_cast<const f32x4*>(a_src + j * a_step + kn);
#pragma unroll
    for (int j = 0; j < VW; ++j) rw[j] = *reinterpret_cast<const f32x4*>(w_src + j * w_step + kn);
    // keep the prefetch ahead of the MFMA block (hipcc otherwise sinks the loads to their
    // consumer, the LDS store after the MFMAs, and the latency is exposed every K-tile)
    __builtin_amdgcn_sched_barrier(0);

    const float* As = smem + cur * STAGE + a_off;
    const float* Ws = smem + cur * STAGE + w_off;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      f32x4 fa[TM], fb[TN];
#pragma unroll
      for (int m = 0; m < TM; ++m) fa[m] = *reinterpret_cast<const f32x4*>(As + m * 32 * LDS_LD + v * 4);
#pragma unroll
      for (int n = 0; n < TN; ++n) fb[n] = *reinterpret_cast<const f32x4*>(Ws + n * 32 * LDS_LD + v * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int n = 0; n < TN; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[m][e], fb[n][e], acc[m][n], 0, 0, 0);
    }
    const int nb = (cur ^ 1) * STAGE;
#pragma unroll
    for (int j = 0; j < VA; ++j) *reinterpret_cast<f32x4*>(a_dst0 + nb + j * RS * LDS_LD) = ra[j];
#pragma unroll
    for (int j = 0; j < VW; ++j) *reinterpret_cast<f32x4*>(w_dst0 + nb + j * RS * LDS_LD) = rw[j];
    __syncthreads();
  }
  epilogue<EPI, TL>(a, acc, g, tm, tn);
}

// Grid = one workgroup per tile.
template <int EPI, class TL>
__global__ __launch_bounds__(TL::NT, TL::OCC) void k_gemm_nt(GemmArgs a) {
  gemm_tile<EPI, TL>(a, blockIdx.x);
}

// ==== bf16x6: the same fp32 GEMM on the bf16 matrix pipe ==================================
// Each fp32 operand is split exactly into three bf16 limbs, x = x0 + x1 + x2 (RNE at each
// step; |x1| <= 2^-8|x|, |x2| <= 2^-16|x|, the last remainder has <= 8 significant bits so
// the split is exact for normal numbers).  The product a*b is then the six limb products of
// degree <= 2: a0b0 + (a0b1 + a1b0) + (a1b1 + a0b2 + a2b0); the dropped a1b2 + a2b1 + a2b2
// are <= 2^-23|ab| (typically ~2^-27), below the fp32 rounding of one fma.  Each limb
// product of two bf16 is exact in fp32 and v_mfma_f32_32x32x16_bf16 accumulates in fp32, so
// the result carries fp32-level error (measured against fp64: tools/x6_accuracy.py) at 6
// bf16 MFMAs = 6 x 32 cycles per 32x32x16 block instead of 8 f32 MFMAs x 64 cycles: 2.67x
// fewer matrix-pipe cycles per f32 MAC.
//
// Weights are split once (amx_split_bf16x3) into a K-tiled image [N][K/16][limb][16], so a
// row's K-tile is 96 contiguous bytes; the fp32 activations are split while they are staged
// into LDS.  BK = 16 fp32 k per K-tile; an LDS row holds [limb0 k0..15 | limb1 | limb2 | 8
// pad] = 56 bf16 = 112 B (28 dwords: the 16-lane groups of ds_read_b128 hit all 64 banks
// once).  Lane l of an MFMA reads row l&31, k-chunk 8*(l>>5) of the limb it needs.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int XBK = 16;  // granule of the weight image: 16 fp32 k per [limb][16] chunk

// LDS row = [limb0 16 | limb1 | limb2] + 8 bf16 pad (56 bf16 = 28 dwords: the 16 rows of a
// ds_read_b128 lane group land on distinct 4-bank slots); BK = 16, double-buffered LDS, one
// barrier per K-tile.
template <int WM_, int WN_, int TM_, int TN_, int OCC_ = 2>
struct TileX6 {
  static constexpr int WM = WM_, WN = WN_, TM = TM_, TN = TN_, OCC = OCC_;
  static constexpr int BK = 16;
  static constexpr int LD = 48 + 8;                            // bf16 per LDS row
  static constexpr int NT = WM * WN * 64;
  static constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  static constexpr int STAGE = (BM + BN) * LD;                 // bf16 of one stage (A + W)
  static constexpr size_t LDS = 2 * STAGE * sizeof(uint16_t);
  static constexpr int NA = BM * (BK / 4);                     // 16-B chunks of the A tile (fp32)
  static constexpr int NW = BN * 6;                            // 16-B chunks of the W tile
  static constexpr int VA = (NA + NT - 1) / NT, VW = (NW + NT - 1) / NT;
  static_assert(LDS <= 160 * 1024, "LDS");
};

// x (4 consecutive k of one row) -> limbs packed as 4 bf16 each
__device__ __forceinline__ void split3(f32x4 x, u32x2& l0, u32x2& l1, u32x2& l2) {
  const bf16x4 h0 = __builtin_convertvector(x, bf16x4);
  const f32x4 r1 = x - __builtin_convertvector(h0, f32x4);  // exact
  const bf16x4 h1 = __builtin_convertvector(r1, bf16x4);
  const f32x4 r2 = r1 - __builtin_convertvector(h1, f32x4);  // exact
  const bf16x4 h2 = __builtin_convertvector(r2, bf16x4);     // exact (<= 8 significant bits)
  l0 = __builtin_bit_cast(u32x2, h0);
  l1 = __builtin_bit_cast(u32x2, h1);
  l2 = __builtin_bit_cast(u32x2, h2);
}

template <int EPI, class TL>
__device__ __forceinline__ void gemm_tile_x6(const GemmArgs& a, int orig) {
  constexpr int BM = TL::BM, TM = TL::TM, TN = TL::TN, VA = TL::VA, VW = TL::VW, LD = TL::LD;
  constexpr int NT = TL::NT, STAGE = TL::STAGE, BK = TL::BK, CPR = BK / 4;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint16_t* const sm = reinterpret_cast<uint16_t*>(smem);
  int g, tm, tn;
  map_tile(a, orig, g, tm, tn);
  const float* __restrict__ Ag = a.A + (long long)g * a.strideA + (long long)tm * BM * a.lda;
  const long long ldw3 = 3LL * a.K;
  const uint16_t* __restrict__ Wg = a.W3 + (long long)g * a.strideW3 + (long long)tn * TL::BN * ldw3;

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int li = lane & 31, lh = lane >> 5;

  // staging maps: A chunk q = t + NT*j -> row q / CPR, k 4*(q % CPR);
  // W chunk q -> row q / 6, 16-B piece p = q % 6, stored in the image's order
  const float* a_src[VA];
  int a_dst[VA];
  bool a_ok[VA];
#pragma unroll
  for (int j = 0; j < VA; ++j) {
    const int q = t + NT * j;
    a_ok[j] = (TL::NA % NT == 0 || j + 1 < VA) ? true : q < TL::NA;  // compile-time true but for a ragged last pass
    const int r = a_ok[j] ? q / CPR : 0, c = q % CPR;
    a_src[j] = Ag + (long long)r * a.lda + 4 * c;
    a_dst[j] = r * LD + c * 4;
  }
  const uint16_t* w_src[VW];
  int w_dst[VW];
  bool w_ok[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    const int q = t + NT * j;
    w_ok[j] = (TL::NW % NT == 0 || j + 1 < VW) ? true : q < TL::NW;
    const int r = w_ok[j] ? q / 6 : 0, p = q % 6;
    w_src[j] = Wg + (long long)r * ldw3 + p * 8;
    w_dst[j] = BM * LD + r * LD + p * 8;
  }

  f32x4 ra[VA];
  u32x4 rw[VW];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = a.K / BK;
  auto load = [&](int kt) {
    kt = kt < nk ? kt : nk - 1;  // past the end: re-read the last tile (branch-free)
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok[j]) ra[j] = *reinterpret_cast<const f32x4*>(a_src[j] + kt * BK);
#pragma unroll
    for (int j = 0; j < VW; ++j)
      if (w_ok[j]) rw[j] = *reinterpret_cast<const u32x4*>(w_src[j] + kt * 48);
  };
  auto publish = [&](int base) {
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok[j]) {
        u32x2 l0, l1, l2;
        split3(ra[j], l0, l1, l2);
        *reinterpret_cast<u32x2*>(sm + base + a_dst[j]) = l0;
        *reinterpret_cast<u32x2*>(sm + base + a_dst[j] + 16) = l1;
        *reinterpret_cast<u32x2*>(sm + base + a_dst[j] + 32) = l2;
      }
#pragma unroll
    for (int j = 0; j < VW; ++j)
      if (w_ok[j]) *reinterpret_cast<u32x4*>(sm + base + w_dst[j]) = rw[j];
  };
  const int a_off = (wm * TM * 32 + li) * LD + lh * 8;
  const int w_off = BM * LD + (wn * TN * 32 + li) * LD + lh * 8;
  auto compute = [&](int base) {
    const uint16_t* As = sm + base + a_off;
    const uint16_t* Ws = sm + base + w_off;
    bf16x8 fa[TM][3], fb[TN][3];
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int l = 0; l < 3; ++l) fa[m][l] = *reinterpret_cast<const bf16x8*>(As + m * 32 * LD + l * 16);
#pragma unroll
    for (int n = 0; n < TN; ++n)
#pragma unroll
      for (int l = 0; l < 3; ++l) fb[n][l] = *reinterpret_cast<const bf16x8*>(Ws + n * 32 * LD + l * 16);
    // small terms first: (a2,b0) (a0,b2) (a1,b1) (a1,b0) (a0,b1) (a0,b0)
    constexpr int PA[6] = {2, 0, 1, 1, 0, 0}, PB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
    for (int p = 0; p < 6; ++p)
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int n = 0; n < TN; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][PA[p]], fb[n][PB[p]], acc[m][n], 0, 0, 0);
  };

  load(0);
  publish(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    load(kt + 1);
    // keep the prefetch ahead of the MFMA block (hipcc otherwise sinks the loads to their
    // consumer, the LDS store after the MFMAs)
    __builtin_amdgcn_sched_barrier(0);
    compute(cur * STAGE);
    publish((cur ^ 1) * STAGE);
    __syncthreads();
  }
  epilogue<EPI, TL>(a, acc, g, tm, tn);
}

template <int EPI, class TL>
__global__ __launch_bounds__(TL::NT, TL::OCC) void k_gemm_x6(GemmArgs a) {
  gemm_tile_x6<EPI, TL>(a, blockIdx.x);
}

// fp32 [g][rows][K] (ld, stride) -> 3-limb bf16 image [g][rows][K/16][3][16]
__global__ void k_split_bf16x3(const float* __restrict__ W, int ldw, long long strideW, int rows, int K,
                               uint16_t* __restrict__ W3, long long strideW3) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // one f32x4 chunk
  const int cpr = K / 4;
  const int g = blockIdx.y;
  if (q >= (long long)rows * cpr) return;
  const int r = (int)(q / cpr), c = (int)(q % cpr) * 4;
  const f32x4 x = *reinterpret_cast<const f32x4*>(W + g * strideW + (long long)r * ldw + c);
  u32x2 l0, l1, l2;
  split3(x, l0, l1, l2);
  uint16_t* dst = W3 + g * strideW3 + (long long)r * 3 * K + (c / XBK) * 48 + (c % XBK);
  *reinterpret_cast<u32x2*>(dst) = l0;
  *reinterpret_cast<u32x2*>(dst + 16) = l1;
  *reinterpret_cast<u32x2*>(dst + 32) = l2;
}



// bias / activation / un-normalisation epilogue of the scaled path; for a hidden layer it also
// reduces the exponents of the rows it wrote (over its columns) into row_exp_out.
template <int EPI, class TL>
__device__ __forceinline__ void epilogue_h3_impl(const GemmArgs& a, f32x16 (&acc)[TL::TM][TL::TN], const int* sExp,
                                                 int g, int tm, int tn);

// EPI_RFF: the accumulators are un-scaled in place (exact powers of two) and handed to the
// shared RFF epilogue (cos, phi rows, fp64 column partials), which reuses the stage LDS
template <int EPI, class TL>
__device__ __forceinline__ void epilogue_h3(const GemmArgs& a, f32x16 (&acc)[TL::TM][TL::TN], const int* sExp, int g,
                                            int tm, int tn) {
  if constexpr (EPI == EPI_RFF) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave / TL::WN, wn = wave % TL::WN, li = lane & 31, lh = lane >> 5;
    const int* wexp = a.w_exp + (long long)g * a.strideWexp;
#pragma unroll
    for (int n = 0; n < TL::TN; ++n) {
      const int ec = wexp[tn * TL::BN + wn * TL::TN * 32 + n * 32 + li] - 2 * HSC;
#pragma unroll
      for (int m = 0; m < TL::TM; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          acc[m][n][e] = __builtin_amdgcn_ldexpf(
              acc[m][n][e], sExp[wm * TL::TM * 32 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh] + ec);
    }
    __syncthreads();  // every wave is done with the stage buffers (and with sExp)
    epilogue<EPI_RFF, TL>(a, acc, g, tm, tn);
  } else {
    epilogue_h3_impl<EPI, TL>(a, acc, sExp, g, tm, tn);
  }
}

template <int EPI, class TL>
__device__ __forceinline__ void epilogue_h3_impl(const GemmArgs& a, f32x16 (&acc)[TL::TM][TL::TN], const int* sExp,
                                                 int g, int tm, int tn) {
  constexpr int BM = TL::BM, BN = TL::BN, TM = TL::TM, TN = TL::TN;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int li = lane & 31, lh = lane >> 5;
  const int lrow0 = wm * TM * 32;                 // tile-local
  const int row0 = tm * BM + lrow0;
  const int col0 = tn * BN + wn * TN * 32;
  const float* bias = a.bias + (long long)g * a.strideBias;
  const int* wexp = a.w_exp + (long long)g * a.strideWexp;
  float* Cg = a.C + (long long)g * a.strideC;
  // row exponents of this lane's 16 rows of block m (rows in groups of 4: ds_read_b128)
  auto row_exps = [&](int m, int (&er)[16]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int4 v = *reinterpret_cast<const int4*>(sExp + lrow0 + m * 32 + 8 * j + 4 * lh);
      er[4 * j] = v.x; er[4 * j + 1] = v.y; er[4 * j + 2] = v.z; er[4 * j + 3] = v.w;
    }
  };
  if constexpr (EPI == EPI_BIAS_ACT) {
    float bv[TN];
    int ec[TN];
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int col = col0 + n * 32 + li;
      bv[n] = bias[col];
      ec[n] = wexp[col] - 2 * HSC;
    }
    int* out = a.row_exp_out ? a.row_exp_out + (long long)g * a.strideRexp : nullptr;
#pragma unroll
    for (int m = 0; m < TM; ++m) {
      int er[16];
      row_exps(m, er);
      uint32_t mx[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) mx[e] = 0u;
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const int col = col0 + n * 32 + li;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = row0 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          float v = __builtin_amdgcn_ldexpf(acc[m][n][e], er[e] + ec[n]) + bv[n];
          if (a.act == AMX_ACT_RELU) v = (v < 0.f) ? 0.f : v;  // keeps NaN, as torch.relu
          Cg[(long long)row * a.ldc + a.col_off + col] = v;
          const uint32_t b = __float_as_uint(v) & 0x7fffffffu;
          mx[e] = mx[e] > b ? mx[e] : b;
        }
      }
      if (out) {
        // max over the 32 columns (lanes li) of the block's 16 rows of this lane: a
        // reduce-scatter butterfly over li bits 4..1 leaves lane li row index li>>1, then
        // one exchange across bit 0
        rs_step<16, 8>(mx, li);
        rs_step<8, 4>(mx, li);
        rs_step<4, 2>(mx, li);
        rs_step<2, 1>(mx, li);
        const uint32_t o = (uint32_t)__builtin_amdgcn_ds_swizzle((int)mx[0], 0x1f | (1 << 10));
        const uint32_t r = mx[0] > o ? mx[0] : o;
        if ((li & 1) == 0) {
          const int e = li >> 1;
          atomicMax(out + row0 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh, exp_of_bits(r));
        }
      }
    }
  } else {  // EPI_UNNORM
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int col = col0 + n * 32 + li;
      if (col < a.n_valid) {
        const float bv = bias[col];
        const float sc = a.scale[col], sh = a.shift[col];
        const int ec = wexp[col] - 2 * HSC;
#pragma unroll
        for (int m = 0; m < TM; ++m) {
          int er[16];
          row_exps(m, er);
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = row0 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
            const float y = __builtin_amdgcn_ldexpf(acc[m][n][e], er[e] + ec) + bv;
            const float prod = y * sc;    // two roundings, as torch's (y*scale)+mean
            Cg[(long long)row * a.ldc + col] = prod + sh;
          }
        }
      }
    }
  }
}

// epilogue of the 16x16x32 form: block (m, n) of the wave holds, per lane, column n*16 + (l&15)
// and rows m*16 + 4(l>>4) + j (j = reg); the row-exponent reduction is a reduce-scatter over
// the 16 column lanes of the lane's MB*4 rows
template <int EPI, class TL>
__device__ __forceinline__ void epilogue_h3_m16(const GemmArgs& a, f32x4 (&acc)[TL::MB][TL::NB], const int* sExp,
                                                int g, int tm, int tn) {
  constexpr int MB = TL::MB, NB = TL::NB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int lc = lane & 15, lq = lane >> 4;
  const int lrow0 = wm * TL::WROWS;
  const int row0 = tm * TL::BM + lrow0;
  const int col0 = tn * TL::BN + wn * TL::WCOLS;
  const float* bias = a.bias + (long long)g * a.strideBias;
  const int* wexp = a.w_exp + (long long)g * a.strideWexp;
  float* Cg = a.C + (long long)g * a.strideC;
  if constexpr (EPI == EPI_RFF) {  // the 32x32 path's RFF epilogue on the 16x16 accumulator layout
    // The tile staged through LDS in passes of RP rows (all of it when it fits the launch's
    // LDS, rff_m16_rows), then one column per thread: the NT / BN threads of a column take the
    // 32-row groups g = part, part + NT / BN, ... (wave-uniform: BN >= 64), each group's phi
    // rows coalesced and its fp64 partial (AMX_RFF_PART_ROWS) summed in row order.
    constexpr int BM = TL::BM, BN = TL::BN, CLD = BN + 4, P = TL::NT / BN, RP = rff_m16_rows(BM, BN);
    static_assert(TL::NT % BN == 0 && BN >= 64 && BM % AMX_RFF_PART_ROWS == 0 && RP % AMX_RFF_PART_ROWS == 0 &&
                      RP % 16 == 0, "RFF epilogue tiles");
    // un-scale in place (exact powers of two) while sExp (in the stage area) is readable
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int4 ev = *reinterpret_cast<const int4*>(sExp + lrow0 + m * 16 + 4 * lq);
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const int ec = wexp[col0 + n * 16 + lc] - 2 * HSC;
        acc[m][n][0] = __builtin_amdgcn_ldexpf(acc[m][n][0], ev.x + ec);
        acc[m][n][1] = __builtin_amdgcn_ldexpf(acc[m][n][1], ev.y + ec);
        acc[m][n][2] = __builtin_amdgcn_ldexpf(acc[m][n][2], ev.z + ec);
        acc[m][n][3] = __builtin_amdgcn_ldexpf(acc[m][n][3], ev.w + ec);
      }
    }
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Cs = smem;  // [RP][CLD] over the stage buffers
    const int t = threadIdx.x, c = t % BN, part = t / BN;
    const int col = tn * BN + c;
    const float bv = a.bias[col];
#pragma unroll
    for (int r0 = 0; r0 < BM; r0 += RP) {
      __syncthreads();  // the stage buffers (or the previous pass) are free
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const int rb = lrow0 + m * 16;  // a 16-row block lies wholly in one pass (RP % 16 == 0)
        if (rb >= r0 && rb < r0 + RP) {
#pragma unroll
          for (int n = 0; n < NB; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              Cs[(rb - r0 + 4 * lq + j) * CLD + wn * TL::WCOLS + n * 16 + lc] = acc[m][n][j];
        }
      }
      __syncthreads();
      constexpr int GP = (RP < BM ? RP : BM) / AMX_RFF_PART_ROWS;  // groups per pass
      for (int gl = part; gl < GP && r0 + gl * AMX_RFF_PART_ROWS < BM; gl += P) {
        const int row0 = tm * BM + r0 + gl * AMX_RFF_PART_ROWS;
        const uint64_t vmask = row_valid_mask(a, row0, AMX_RFF_PART_ROWS);
        double csum = 0.0;
#pragma unroll 8
        for (int i = 0; i < AMX_RFF_PART_ROWS; ++i) {
          const float z = Cs[(gl * AMX_RFF_PART_ROWS + i) * CLD + c] + bv;  // nn.Linear: x W^T + b
          const float phi = rff_cos(z) * a.rff_scale;                       // torch.cos(.) * np.sqrt(2/F)
          a.C[(long long)(row0 + i) * a.ldc + col] = phi;
          csum += ((vmask >> i) & 1u) ? (double)phi : 0.0;
        }
        a.col_partials[(long long)(row0 / AMX_RFF_PART_ROWS) * a.N + col] = csum;
      }
    }
    return;
  }
  if constexpr (EPI == EPI_BIAS_ACT) {
    float bv[NB];
    int ec[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const int col = col0 + n * 16 + lc;
      bv[n] = bias[col];
      ec[n] = wexp[col] - 2 * HSC;
    }
    uint32_t mx[MB * 4];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int4 ev = *reinterpret_cast<const int4*>(sExp + lrow0 + m * 16 + 4 * lq);
      const int er[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) mx[m * 4 + j] = 0u;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const int col = col0 + n * 16 + lc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = row0 + m * 16 + 4 * lq + j;
          float v = __builtin_amdgcn_ldexpf(acc[m][n][j], er[j] + ec[n]) + bv[n];
          if (a.act == AMX_ACT_RELU) v = (v < 0.f) ? 0.f : v;  // keeps NaN, as torch.relu
          Cg[(long long)row * a.ldc + a.col_off + col] = v;
          const uint32_t b = __float_as_uint(v) & 0x7fffffffu;
          mx[m * 4 + j] = mx[m * 4 + j] > b ? mx[m * 4 + j] : b;
        }
      }
    }
    if (a.row_exp_out) {
      int* out = a.row_exp_out + (long long)g * a.strideRexp;
      if constexpr (MB * 4 == 16 || MB * 4 == 32) {
        // reduce-scatter over the 16 column lanes (bits 3..0 of lc): lane lc keeps the PER
        // values of flat indices PER*lc .. PER*lc+PER-1 (flat index = m*4 + j)
        constexpr int NV = MB * 4, PER = NV / 16;
        rs_step<8, NV / 2>(mx, lc);
        rs_step<4, NV / 4>(mx, lc);
        rs_step<2, NV / 8>(mx, lc);
        rs_step<1, NV / 16>(mx, lc);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int i = PER * lc + u, m = i >> 2, j = i & 3;
          atomicMax(out + row0 + m * 16 + 4 * lq + j, exp_of_bits(mx[u]));
        }
      } else {
        // any MB: per 16-row block, reduce-scatter the lane's 4 row values over lc bits 3, 2
        // (value j = 2 bit3 + bit2 remains), then a full max over bits 1, 0
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          uint32_t q4[4] = {mx[m * 4], mx[m * 4 + 1], mx[m * 4 + 2], mx[m * 4 + 3]};
          rs_step<8, 2>(q4, lc);
          rs_step<4, 1>(q4, lc);
          uint32_t o = (uint32_t)__builtin_amdgcn_ds_swizzle((int)q4[0], 0x1f | (2 << 10));
          q4[0] = q4[0] > o ? q4[0] : o;
          o = (uint32_t)__builtin_amdgcn_ds_swizzle((int)q4[0], 0x1f | (1 << 10));
          q4[0] = q4[0] > o ? q4[0] : o;
          if ((lc & 3) == 0)
            atomicMax(out + row0 + m * 16 + 4 * lq + ((lc >> 3) & 1) * 2 + ((lc >> 2) & 1), exp_of_bits(q4[0]));
        }
      }
    }
  } else {  // EPI_UNNORM
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const int col = col0 + n * 16 + lc;
      if (col < a.n_valid) {
        const float bv = bias[col];
        const float sc = a.scale[col], sh = a.shift[col];
        const int ec = wexp[col] - 2 * HSC;
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          const int4 ev = *reinterpret_cast<const int4*>(sExp + lrow0 + m * 16 + 4 * lq);
          const int er[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = row0 + m * 16 + 4 * lq + j;
            const float y = __builtin_amdgcn_ldexpf(acc[m][n][j], er[j] + ec) + bv;
            const float prod = y * sc;    // two roundings, as torch's (y*scale)+mean
            Cg[(long long)row * a.ldc + col] = prod + sh;
          }
        }
      }
    }
  }
}

// One output tile (logical id `tile`, see map_tile; or, stream-K, the K-tiles [kb, ke) of it:
// segment seg of nseg) of the f16x3 GEMM; the caller runs the timer hooks.
template <int EPI, class TL>
__device__ __forceinline__ void h3_tile(const GemmArgs& a, int tile, int kb, int ke, int seg, int nseg) {
  constexpr int BM = TL::BM, TM = TL::TM, TN = TL::TN, VA = TL::VA, VW = TL::VW, LD = TL::LD;
  constexpr int NT = TL::NT, STAGE = TL::STAGE;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint16_t* const sm = reinterpret_cast<uint16_t*>(smem);
  int* sExp = reinterpret_cast<int*>(sm + TL::SEXP);
  int g, tm, tn;
  tile_coords(a, tile, g, tm, tn);
  const float* __restrict__ Ag = a.A + (long long)g * a.strideA + (long long)tm * BM * a.lda;
  const float* __restrict__ Ag0 = a.A + (long long)tm * BM * a.lda;  // group 0: the shared K slice
  const long long ldw2 = 2LL * a.K;
  const uint16_t* __restrict__ Wg = a.W2 + (long long)g * a.strideW2 + (long long)tn * TL::BN * ldw2;

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int li = lane & 31, lh = lane >> 5;

  // row exponents of the tile's A rows: max over the slices this launch reads
  {
    const int* re = a.row_exp + (long long)g * a.strideRexp + (long long)tm * BM;
    const long long slot = (long long)a.tiles_m * BM;  // slot stride = padded rows
    for (int r = t; r < BM; r += NT) {
      int e = -100;
      for (int s = 0; s < a.rexp_slots; ++s) {
        const int v = re[s * slot + r];
        e = v > e ? v : e;
      }
      sExp[r] = e;
    }
  }
  __syncthreads();
  H3_STAMP(a, 1);

  // staging maps: A chunk q = t + NT*j -> row q/CPR, k 4*(q%CPR); W chunk q -> row q/CPR,
  // 16-B piece q%CPR (the image's [granule][limb][16] order is the LDS row's order)
  constexpr int CPR = TL::CPR, NSUB = TL::NSUB, BK = TL::BK;
  int a_src[VA];  // element offsets from the tile's first row (group g, or group 0 below k_shared)
  int a_dst[VA], a_sh[VA];
  bool a_ok[VA];
  const int nks = a.k_shared / BK;
#pragma unroll
  for (int j = 0; j < VA; ++j) {
    const int q = t + NT * j;
    a_ok[j] = (TL::NA % NT == 0 || j + 1 < VA) ? true : q < TL::NA;
    int r = a_ok[j] ? q / CPR : 0;
    const int c = q % CPR;
    if constexpr (TL::AMAP && CPR == 8)  // chunks q>>5 -> 4 rows; lanes 0-7 r, 8-15 r+2, 16-23 r+1, 24-31 r+3
      r = a_ok[j] ? (q >> 5) * 4 + ((q >> 3) & 1) * 2 + ((q >> 4) & 1) : 0;
    a_src[j] = r * a.lda + 4 * c;
    a_dst[j] = r * LD + (c >> 2) * 32 + (c & 3) * 4;
    a_sh[j] = HSC - sExp[r];
  }
  int w_off_b[VW];  // byte offsets from the tile's first weight row
  int w_dst[VW];
  bool w_ok[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    const int q = t + NT * j;
    w_ok[j] = (TL::NW % NT == 0 || j + 1 < VW) ? true : q < TL::NW;
    const int r = w_ok[j] ? q / CPR : 0, p = q % CPR;
    w_off_b[j] = (int)(((long long)r * ldw2 + p * 8) * 2);
    w_dst[j] = BM * LD + r * LD + p * 8;
  }

  // buffer loads: SGPR descriptors for the tile's A panel (group g and group 0) and W panel, a
  // per-thread byte offset and the K-tile's byte offset in an SGPR -- no 64-bit address VALU in
  // the K loop (and 4 VGPRs fewer than per-thread W pointers: the 256 x 256 tile's 44 B of
  // scratch went with them)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Ag), 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsA0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Ag0), 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Wg), 0, 0x7ffffff0, 0x00020000);
  // AFF: chunk j = chunk 0 + j * RSTEP rows (the plain map of the 16x16x32 tiles)
  constexpr bool AFF = H3_AFFINE && TL::M16 && !TL::AMAP && TL::NA % NT == 0 && TL::NW % NT == 0;
  constexpr int RSTEP = NT / CPR;
  auto gA = [&](int j, int kt) -> f32x4 {
    if constexpr (AFF)
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           kt < nks ? rsA0 : rsA, a_src[0] * 4, (kt * BK + j * RSTEP * a.lda) * 4, 0));
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(kt < nks ? rsA0 : rsA, a_src[j] * 4,
                                                                          kt * BK * 4, 0));
  };
  auto gW = [&](int j, int kt) -> u32x4 {
    if constexpr (AFF)
      return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rsW, w_off_b[0], kt * 2 * BK * 2 + (int)(j * RSTEP * ldw2 * 2), 0));
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsW, w_off_b[j], kt * 2 * BK * 2, 0));
  };
  auto adst = [&](int j) { return AFF ? a_dst[0] + j * RSTEP * LD : a_dst[j]; };
  auto wdst = [&](int j) { return AFF ? w_dst[0] + j * RSTEP * LD : w_dst[j]; };
  f32x4 ra[TL::DEEPA ? 2 : 1][VA];  // A stage registers (DEEPA: the sets of tiles t+1 and t+2)
  u32x4 rw[VW];
  constexpr int MB = TL::MB, NB = TL::NB;  // 16x16 blocks of the M16 form
  using AccT = std::conditional_t<TL::M16, f32x4[MB][NB], f32x16[TM][TN]>;
  AccT acc;
  if constexpr (TL::M16) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  }

  const int nk = a.K / BK;
  auto load_a = [&](auto set, int kt) {
    kt = kt < nk ? kt : nk - 1;  // past the end: re-read the last tile (branch-free)
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok[j]) ra[decltype(set)::value][j] = gA(j, kt);
  };
  auto load_w = [&](int kt) {
    kt = kt < nk ? kt : nk - 1;
#pragma unroll
    for (int j = 0; j < VW; ++j)
      if (w_ok[j]) rw[j] = gW(j, kt);
  };
  // the prologue's loads in the K loop's piece order (A chunks, then W chunks; each pinned by a
  // sched_barrier).  The compiler's waits at the loop head merge the prologue's pending-load
  // order with the back edge's: left to the scheduler, the prologue issued them in reverse (A
  // chunk 0 youngest), and the first publish of EVERY K-tile then waited vmcnt(0) -- for all
  // of the previous tile's loads, the W chunks issued just before the barrier included.
  // staging piece q: an A chunk or a W chunk (SPREAD with VA == VW alternates them, so every
  // m-block carries one A split; otherwise the A chunks first)
  constexpr bool ALT = TL::SPREAD && VA == VW;
  auto piece_a = [](int q) { return ALT ? (q & 1) == 0 : q < VA; };
  auto piece_j = [](int q) { return ALT ? q >> 1 : (q < VA ? q : q - VA); };
  auto load = [&](int kt) {
    kt = kt < nk ? kt : nk - 1;
#pragma unroll
    for (int q = 0; q < VA + VW; ++q) {
      const int j = piece_j(q);
      if (piece_a(q)) {
        if (a_ok[j]) ra[0][j] = gA(j, kt);
      } else {
        if (w_ok[j]) rw[j] = gW(j, kt);
      }
      if constexpr (H3_ORDERED_LOADS) __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto publish = [&](int base) {  // A from set 0
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok[j]) {
        f32x4 x = ra[0][j];
#if H3_EXP & 2
        const u32x4 xb = __builtin_bit_cast(u32x4, x);
        const u32x2 l0 = {xb[0], xb[1]}, l1 = {xb[2], xb[3]};
#else
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_ldexpf(x[i], a_sh[j]);
        u32x2 l0, l1;
        split2(x, l0, l1);
#endif
        *reinterpret_cast<u32x2*>(sm + base + adst(j)) = l0;
        *reinterpret_cast<u32x2*>(sm + base + adst(j) + 16) = l1;
      }
#pragma unroll
    for (int j = 0; j < VW; ++j)
      if (w_ok[j]) *reinterpret_cast<u32x4*>(sm + base + wdst(j)) = rw[j];
  };
  // one staging piece (SPLIT): publish A/W chunk j of the registered tile, then reload chunk j
  // of tile kt (clamped as load()); DEEPA: A chunk j of register set `set`, reloaded with tile
  // kt + 1 (two tiles ahead of the W operand's one)
  auto piece = [&](int q, int base, int kt, auto set) {
    constexpr int SA = decltype(set)::value;
    const int kta = TL::DEEPA ? (kt + 1 < nk ? kt + 1 : nk - 1) : (kt < nk ? kt : nk - 1);
    kt = kt < nk ? kt : nk - 1;
    if (q >= VA + VW) return;
    if (piece_a(q)) {
      const int j = piece_j(q);
      if (a_ok[j]) {
        f32x4 x = ra[SA][j];
#if H3_EXP & 2
        const u32x4 xb = __builtin_bit_cast(u32x4, x);
        const u32x2 l0 = {xb[0], xb[1]}, l1 = {xb[2], xb[3]};
#else
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_ldexpf(x[i], a_sh[j]);
        u32x2 l0, l1;
        split2(x, l0, l1);
#endif
        *reinterpret_cast<u32x2*>(sm + base + adst(j)) = l0;
        *reinterpret_cast<u32x2*>(sm + base + adst(j) + 16) = l1;
#if !(H3_EXP & 1)
        ra[SA][j] = gA(j, kta);
#endif
      }
    } else {
      const int j = piece_j(q);
      if (w_ok[j]) {
        *reinterpret_cast<u32x4*>(sm + base + wdst(j)) = rw[j];
#if !(H3_EXP & 1)
        rw[j] = gW(j, kt);
#endif
      }
    }
  };
  const int a_off = (wm * TM * 32 + li) * LD + lh * 8;
  const int w_off = BM * LD + (wn * TN * 32 + li) * LD + lh * 8;
  // M16: lane l reads row l&15 of a block, k = 8(l>>4)..+7 = granule l>>5, half (l>>4)&1
  const int koff16 = (lane >> 5) * 32 + ((lane >> 4) & 1) * 8;
  const int a_off16 = (wm * TL::WROWS + (lane & 15)) * LD + koff16;
  const int w_off16 = BM * LD + (wn * TL::WCOLS + (lane & 15)) * LD + koff16;
  f16x8 gb[NB][2], ga[2][2];
  // the first fragments of the K-tile in buffer `base` (EARLY: issued right after the barrier,
  // ahead of the LDS writes of the next tile, so the first MFMAs do not wait for those writes)
  auto frag0 = [&](int base) {
    if constexpr (TL::M16) {
      const uint16_t* As = sm + base + a_off16;
      const uint16_t* Ws = sm + base + w_off16;
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int l = 0; l < 2; ++l) gb[n][l] = *reinterpret_cast<const f16x8*>(Ws + n * 16 * LD + l * 16);
#pragma unroll
      for (int l = 0; l < 2; ++l) ga[0][l] = *reinterpret_cast<const f16x8*>(As + l * 16);
    }
  };
  int split_base = 0, split_kt = 0;  // SPLIT: where compute16's pieces publish / what they load
  auto compute16 = [&](int base, auto set) {  // set: the A register set its pieces publish (DEEPA)
    if constexpr (TL::M16) {
    const uint16_t* As = sm + base + a_off16;
    if constexpr (!TL::EARLY) frag0(base);
    // the reads of block m+1 are pinned ahead of block m's MFMAs (sched_barrier): hipcc
    // otherwise reloads one fragment register at a time and waits lgkmcnt(0) per MFMA group
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      if (m + 1 < MB) {
#pragma unroll
        for (int l = 0; l < 2; ++l)
          ga[(m + 1) & 1][l] = *reinterpret_cast<const f16x8*>(As + (m + 1) * 16 * LD + l * 16);
      }
      if constexpr (TL::PIN && !TL::SPREAD) __builtin_amdgcn_sched_barrier(0);
      constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};  // small terms first
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int n = 0; n < NB; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ga[m & 1][PA[p]], gb[n][PB[p]], acc[m][n], 0, 0, 0);
      if constexpr (TL::PIN && !TL::SPREAD) __builtin_amdgcn_sched_barrier(0);
      if constexpr (TL::SPREAD) {
        // one wave per SIMD: no partner wave covers the staging work, so it is interleaved into
        // the block's MFMA stream (sched_group_barrier: MFMA / DS read / VALU / DS write / VMEM)
        constexpr int PPB = (VA + VW + MB - 1) / MB;
#pragma unroll
        for (int q = m * PPB; q < (m + 1) * PPB; ++q) piece(q, split_base, split_kt, set);
        constexpr int NMF = 3 * NB;
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
#pragma unroll
        for (int i = 0; i < PPB; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF - 14 - 2 * PPB, 0);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (TL::SPLIT) {
        piece(m, split_base, split_kt, set);
        if (m == MB - 1) {
#pragma unroll
          for (int q = MB; q < VA + VW; ++q) piece(q, split_base, split_kt, set);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    }
  };
  auto compute = [&](int base) {
    if constexpr (TL::M16) {
      compute16(base, std::integral_constant<int, 0>{});
      return;
    } else {
    const uint16_t* As = sm + base + a_off;
    const uint16_t* Ws = sm + base + w_off;
    // m-outer order: the W fragments of the granule stay in registers, the A fragments of
    // block m+1 are read while block m's 3*TN MFMAs run (fewer live fragment registers than
    // reading the whole granule up front; each accumulator still sees the same sequence)
    f16x8 fb[TN][2], fa[2][2];
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {
#pragma unroll
      for (int n = 0; n < TN; ++n)
#pragma unroll
        for (int l = 0; l < 2; ++l)
          fb[n][l] = *reinterpret_cast<const f16x8*>(Ws + n * 32 * LD + sub * 32 + l * 16);
#pragma unroll
      for (int l = 0; l < 2; ++l) fa[0][l] = *reinterpret_cast<const f16x8*>(As + sub * 32 + l * 16);
#pragma unroll
      for (int m = 0; m < TM; ++m) {
        if (m + 1 < TM) {
#pragma unroll
          for (int l = 0; l < 2; ++l)
            fa[(m + 1) & 1][l] = *reinterpret_cast<const f16x8*>(As + (m + 1) * 32 * LD + sub * 32 + l * 16);
        }
        if constexpr (TL::PIN) __builtin_amdgcn_sched_barrier(0);
        // small terms first: (a1,b0) (a0,b1) (a0,b0)
        constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int n = 0; n < TN; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[m & 1][PA[p]], fb[n][PB[p]], acc[m][n], 0, 0, 0);
        if constexpr (TL::PIN) __builtin_amdgcn_sched_barrier(0);
      }
    }
    }
  };

  auto finish = [&](AccT& ac) {
    if constexpr (TL::M16) {
      // the row exponents lived in stage buffer 1 during the prologue; re-read them into LDS
      __syncthreads();
      sExp = reinterpret_cast<int*>(sm);
      const int* re = a.row_exp + (long long)g * a.strideRexp + (long long)tm * BM;
      const long long slot = (long long)a.tiles_m * BM;
      for (int r = t; r < BM; r += NT) {
        int e = -100;
        for (int s2 = 0; s2 < a.rexp_slots; ++s2) {
          const int v = re[s2 * slot + r];
          e = v > e ? v : e;
        }
        sExp[r] = e;
      }
      __syncthreads();
      epilogue_h3_m16<EPI, TL>(a, ac, sExp, g, tm, tn);
    } else {
      epilogue_h3<EPI, TL>(a, ac, sExp, g, tm, tn);
    }
  };
  if constexpr (TL::DEEPA) {
    // K-tiles [kb, ke); tile x's A in register set (x - kb) & 1, loaded two tiles ahead
    load(kb);
    publish(0);
    load_a(std::integral_constant<int, 1>{}, kb + 1);
    load_w(kb + 1);
    load_a(std::integral_constant<int, 0>{}, kb + 2);
    H3_STAMP(a, 2);
    auto kstep = [&](int kt, auto par) {  // buffer par; pieces publish tile kt+1 from set par^1
      constexpr int P = decltype(par)::value;
      __syncthreads();  // tile kt visible in buffer P; buffer P^1 (tile kt-1) fully read
      frag0(P * STAGE);
      __builtin_amdgcn_sched_barrier(0);
      split_base = (P ^ 1) * STAGE;
      split_kt = kt + 2;
      compute16(P * STAGE, std::integral_constant<int, P ^ 1>{});
    };
    for (int kt = kb; kt < ke; kt += 2) {
      kstep(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < ke) kstep(kt + 1, std::integral_constant<int, 1>{});
    }
    H3_STAMP(a, 3);
    if constexpr (EPI == EPI_UNNORM) {
      if (nseg > 1) {
        __syncthreads();  // the stage buffers are free: one int of LDS for the last-arriver flag
        if (!split_combine<TL>(a, acc, tile, seg, nseg, reinterpret_cast<int*>(smem) + BM + 4)) return;
      }
    }
    finish(acc);
#if H3_TRACE
    H3_STAMP(a, 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    H3_STAMP(a, 5);
#endif
    return;
  }
  if constexpr (TL::LATE) {
    // K-tiles [kb, ke) of this workgroup (all of them unless the tile is split)
    load(kb);
    publish(0);
    load(kb + 1);
    H3_STAMP(a, 2);
    for (int kt = kb; kt < ke; ++kt) {
      const int cur = (kt - kb) & 1;
      __syncthreads();  // tile kt visible in buffer cur; buffer cur^1 (tile kt-1) fully read
      if constexpr (TL::EARLY) {
        frag0(cur * STAGE);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (TL::SPLIT) {  // tile kt+1's publish and tile kt+2's loads run inside compute
        split_base = (cur ^ 1) * STAGE;
        split_kt = kt + 2;
        compute(cur * STAGE);
        continue;
      }
      publish((cur ^ 1) * STAGE);  // tile kt+1 (past the end: a harmless re-publish)
      load(kt + 2);
      __builtin_amdgcn_sched_barrier(0);
      compute(cur * STAGE);
    }
    H3_STAMP(a, 3);
    // (the 256 x 256 hidden tile is launched one tile per workgroup only: no combine code, whose
    // registers it cannot spare)
    if constexpr (TL::M16 && (EPI == EPI_UNNORM || (EPI == EPI_BIAS_ACT && !(BM == 256 && TL::BN == 256)))) {
      if (nseg > 1) {
        __syncthreads();  // the stage buffers are free: one int of LDS for the last-arriver flag
        if (!split_combine<TL>(a, acc, tile, seg, nseg, reinterpret_cast<int*>(smem) + BM + 4)) return;
      }
    }
    finish(acc);
#if H3_TRACE
    H3_STAMP(a, 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    H3_STAMP(a, 5);
#endif
    return;
  }
  load(0);
  publish(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    load(kt + 1);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the MFMA block
    compute(cur * STAGE);
    publish((cur ^ 1) * STAGE);
    __syncthreads();
  }
  finish(acc);
}

// a.streamk (LATE M16 UNNORM tiles): one workgroup per CU; the workgroups of one XCD take
// consecutive virtual ids v (xcd_logical) and v runs the K-tiles [v U / G, (v + 1) U / G) of
// the U = tiles x nk units in logical tile order (tile_n fastest, then tile_m: an XCD's
// workgroups share A row panels and one member's weight panels in its L2) -- one, two or three
// segments of consecutive tiles -- and the tiles' segments are combined in K order
// (split_combine).  Otherwise one tile per workgroup (map_tile's XCD-contiguous order).
template <int EPI, class TL>
__global__ __launch_bounds__(TL::NT, TL::OCC) void k_gemm_h3(GemmArgs a) {
  if (a.timer_role == 1 && blockIdx.x == 0 && threadIdx.x == 0) a.timer[0] = __builtin_amdgcn_s_memrealtime();
  H3_STAMP(a, 0);
  const int nk = a.K / TL::BK;
  if (a.streamk) {
    const long long U = (long long)a.tiles_m * a.tiles_n * a.groups * nk, G = gridDim.x;
    const int v = xcd_logical((int)G, (int)blockIdx.x);
    long long u = (long long)v * U / G;
    const long long uend = ((long long)v + 1) * U / G;
    while (u < uend) {
      const int tile = (int)(u / nk), kb = (int)(u - (long long)tile * nk);
      const int ke = (uend - u) < (long long)(nk - kb) ? kb + (int)(uend - u) : nk;
      const long long u0 = (long long)tile * nk;
      const int wf = (int)(((u0 + 1) * G - 1) / U), wl = (int)(((u0 + nk) * G - 1) / U);  // its workgroups
      h3_tile<EPI, TL>(a, tile, kb, ke, v - wf, wl - wf + 1);
      u += ke - kb;
      __syncthreads();  // LDS reuse by the next segment
    }
  } else {
    h3_tile<EPI, TL>(a, xcd_logical(a.tiles_m * a.tiles_n * a.groups, (int)blockIdx.x), 0, nk, 0, 1);
  }
  if (a.timer_role == 2) gemm_timer_end(a);
}

// fp32 [g][rows][K] -> scaled 2-limb f16 image [g][rows][K/16][2][16] + row exponents
// [g][rows]: one wave per row (max |w| over K, then the split)
__global__ __launch_bounds__(256) void k_split_f16x2(const float* __restrict__ W, int ldw, long long strideW,
                                                     int rows, int K, uint16_t* __restrict__ W2, long long strideW2,
                                                     int* __restrict__ w_exp, long long strideWexp) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.y;
  if (r >= rows) return;
  const float* src = W + g * strideW + (long long)r * ldw;
  uint32_t mx = 0;
  for (int c = 4 * lane; c < K; c += 256) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(src + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t b = __float_as_uint(x[i]) & 0x7fffffffu;
      mx = mx > b ? mx : b;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)mx, off);
    mx = mx > o ? mx : o;
  }
  const int e = exp_of_bits(mx);
  if (lane == 0) w_exp[g * strideWexp + r] = e;
  uint16_t* dst_row = W2 + g * strideW2 + (long long)r * 2 * K;
  for (int c = 4 * lane; c < K; c += 256) {
    f32x4 x = *reinterpret_cast<const f32x4*>(src + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_ldexpf(x[i], HSC - e);
    u32x2 l0, l1;
    split2(x, l0, l1);
    uint16_t* dst = dst_row + (c / 16) * 32 + (c % 16);
    *reinterpret_cast<u32x2*>(dst) = l0;
    *reinterpret_cast<u32x2*>(dst + 16) = l1;
  }
}

// row exponents of A's first K columns (the x0 slice) into slot 0 of row_exp, slots
// 1..n_slots-1 reset to -100 (the hidden epilogues max into them): one wave per row
__global__ __launch_bounds__(256) void k_row_exp(const float* __restrict__ A, int lda, long long strideA, int rows,
                                                 int K, int* __restrict__ row_exp, long long strideRexp, int n_slots) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.y;
  if (r >= rows) return;
  const float* src = A + g * strideA + (long long)r * lda;
  uint32_t mx = 0;
  for (int c = lane; c < K; c += 64) {
    const uint32_t b = __float_as_uint(src[c]) & 0x7fffffffu;
    mx = mx > b ? mx : b;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)mx, off);
    mx = mx > o ? mx : o;
  }
  int* re = row_exp + g * strideRexp + r;
  if (lane < n_slots) re[(long long)lane * rows] = lane == 0 ? exp_of_bits(mx) : -100;
}

// The tiles the launchers pick (chosen by same-process A/B runs in round 1: DESIGN.md §3.0,
// profiles/r01_h3_*.txt):
//   hidden layers, grid >= one WG per CU: 256x256, BK 32, 8 waves of 128x64 on 16x16x32,
//     write-after-barrier with pinned / early fragment reads and split staging (160 KB LDS)
//   otherwise (and the RFF features): 128x128, BK 32, 4 waves of 64x64 on 32x32x16
//   output layer S <= 224: 128x224, 14 waves of 64x32 on 16x16x32 (same schedule);
//     S in (224, 256]: 128x256, 8 waves of 64x64
using H256 = TileH3<2, 4, 4, 2, 2, 2, true, true, true, 0, 0, true, true, true>;
// 4 waves of 128 x 128, one per SIMD (H3_W4 A/B): 192 MFMAs and 32 fragment reads per wave and
// K-tile, the 16 staging pieces two behind each m-block
using H256w4 = TileH3<2, 2, 4, 4, 1, 2, true, true, true, 0, 0, true, true, true, false, true>;
// row-block tiles for the strong-scaling lane counts (rows = 32 RB, 4 members: a 256-workgroup
// grid for every RB): hidden RB x 256 (8 waves of RB/2 x 64), output RB x 112 / RB x 128
// (RB/32 waves of 32 x 112 or 32 x 128), same schedule as H256
template <int MB> using HRow = TileH3<2, 4, 1, 1, 2, 2, true, true, true, MB, 4, true, true, true>;
template <int RW, int NBO> using HOut = TileH3<RW, 1, 1, 1, 2, 2, true, true, true, 2, NBO, true, true, true>;
using H128k32 = TileH3<2, 2, 2, 2, 2, 2>;
// the RFF pass's 128 x 128 tile at three workgroups per CU: BK 16 (41.5 KB of stage buffers),
// the epilogue staged in two 64-row passes (RFF_OCC3)
using H128rff3 = TileH3<2, 2, 2, 2, 3, 1>;
// RFF features at row counts whose 128 x 128 tiles fill less than the CUs (the 4- and 8-GPU
// strong-scaling shares): 128 x 64, 4 waves of 32 x 64 (half the work per workgroup, twice
// the workgroups; the same column-partial layout [rows / 128][F])
using H128x64k32 = TileH3<4, 1, 1, 2, 2, 2>;
using H128 = TileH3<2, 2, 2, 2>;  // K not a multiple of 32 (BK 16)
// RFF features on 160-row tiles (32-row column partials, AMX_RFF_PART_ROWS): 160 x 256, 8 waves
// of 80 x 64 (the 5120-lane hidden tile's waves), one per CU -- 40 960 rows x 512 features are
// 512 tiles, exactly two rounds (the 128 x 128 tiles at three per CU: 1280 in 1.67 rounds):
// 88.5 -> 76.2 us under rocprofv3, same box (profiles/r05e_rff160_ab.txt).  (A 160 x 64 tile,
// 4 waves of 80 x 32 at two per CU -- 5120 rows in one round of 256 tiles -- took 25.1 us
// against the 128 x 64 tile's 23.1 and was dropped.)
using H160x256r = TileH3<2, 4, 1, 1, 1, 2, true, true, true, 5, 4, true, true, true>;
using H128x224 = TileH3<2, 7, 2, 1, 4, 2, true, true, true, 0, 0, true, true, true, true>;  // + DEEPA (-2 %)
// 80 x 224 output tiles, 7 waves of 80 x 32 (16x16x32 form, split schedule): one tile per CU when
// groups * rows / 80 == CUs (5120 lanes x 4 members: the N = 4 / 8 per-rank shares) -- no
// stream-K partial tiles, the A panel read once
using H80x224 = TileH3<1, 7, 1, 1, 1, 2, true, true, true, 5, 2, true, true, true, true>;  // + DEEPA


using H128x224k16 = TileH3<2, 7, 2, 1, 4>;  // K not a multiple of 32
using H128x256 = TileH3<2, 4, 2, 2, 2, 2, true, true, true, 0, 0, true, true, true>;
// small-row tiles (the reference-semantics sampler: a few hundred lanes, or 128 per member when
// each lane runs its own member only): 128 x 64 hidden tiles (4 waves of 64 x 32) and 128 x 32
// output tiles (4 waves of 32 x 32), stream-K over up to one workgroup per CU (small_plan) --
// the weight panels read once per K range, 8-32 KB partial tiles per segment
// 8 waves (two per SIMD: one wave's staging overlaps the other's MFMAs) when a member has one
// 128-row tile (the member-blocked sampler's 512 lanes: forward 75 -> 68 us), else 4 waves
// (256+ rows: 85 vs 90 us at 1024 lanes; profiles/r06y_small_tile_waves_ab.txt)
using HS64 = TileH3<2, 2, 1, 1, 2, 2, true, true, true, 4, 2, true, true, true>;
using HS64w8 = TileH3<4, 2, 1, 1, 2, 2, true, true, true, 2, 2, true, true, true>;
using HS32 = TileH3<4, 1, 1, 1, 2, 2, true, true, true, 2, 2, true, true, true>;
using HS32w8 = TileH3<8, 1, 1, 1, 2, 2, true, true, true, 1, 2, true, true, true>;

using X128 = TileX6<2, 2, 2, 2>;        // 128x128, 4 waves of 64x64 (57 KB): 2 WGs / CU
using X256 = TileX6<2, 4, 4, 2>;        // 256x256, 8 waves of 128x64 (115 KB): 1 WG / CU
using X128x224 = TileX6<2, 7, 2, 1, 4>; // output layer (S <= 224), 14 waves of 64x32

using T128 = Tile<2, 2, 2, 2>;          // 128x128, 256 threads, 2 WGs / CU
using T128x224 = Tile<4, 1, 1, 7>;      // 128x224, 256 threads, wave 32x224 (output layer, S <= 224)

// workgroups of a tile shape resident on the context's device at once
int resident_wgs(const amx_ctx* ctx, size_t lds, int nt, int occ) {
  const int by_lds = (int)((160 * 1024) / lds);
  const int by_waves = (occ * 4) / (nt / 64);
  const int per_cu = by_lds < by_waves ? by_lds : by_waves;
  return (per_cu < 1 ? 1 : per_cu) * ctx->n_cus;
}

template <int EPI, class TL>
int launch_nt(GemmArgs& a, hipStream_t stream) {
  a.tiles_m = a.rows / TL::BM;
  a.tiles_n = a.N / TL::BN;
  const int nwg = a.tiles_m * a.tiles_n * a.groups;
  if (nwg == 0) return AMX_OK;
  constexpr size_t lds = (EPI == EPI_RFF && TL::LDS < rff_epi_lds(TL::BM, TL::BN)) ? rff_epi_lds(TL::BM, TL::BN) : TL::LDS;
  hipLaunchKernelGGL((k_gemm_nt<EPI, TL>), dim3(nwg), dim3(TL::NT), lds, stream, a);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

template <int EPI, class TL>
int launch_x6(GemmArgs& a, hipStream_t stream) {
  a.tiles_m = a.rows / TL::BM;
  a.tiles_n = a.N / TL::BN;
  const int nwg = a.tiles_m * a.tiles_n * a.groups;
  if (nwg == 0) return AMX_OK;
  // the RFF epilogue stages the 128x(128+4) f32 tile through LDS (67.6 KB)
  constexpr size_t lds = (EPI == EPI_RFF && TL::LDS < rff_epi_lds(TL::BM, TL::BN)) ? rff_epi_lds(TL::BM, TL::BN) : TL::LDS;
  hipLaunchKernelGGL((k_gemm_x6<EPI, TL>), dim3(nwg), dim3(TL::NT), lds, stream, a);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

template <int EPI, class TL>
int launch_h3(GemmArgs& a, hipStream_t stream) {
  a.tiles_m = a.rows / TL::BM;
  a.tiles_n = a.N / TL::BN;
  const int tiles = a.tiles_m * a.tiles_n * a.groups;
  const int nwg = a.streamk ? a.streamk : tiles;  // stream-K: a.streamk workgroups
  if (tiles == 0) return AMX_OK;
  // (the three-per-CU RFF tile stages its epilogue in two 64-row passes, the M16 tiles in
  // passes of rff_m16_rows)
  constexpr size_t rff_lds = TL::M16      ? rff_epi_lds(rff_m16_rows(TL::BM, TL::BN), TL::BN)
                             : TL::OCC >= 3 ? rff_epi_lds(TL::BM / 2, TL::BN)
                                            : rff_epi_lds(TL::BM, TL::BN);
  constexpr size_t lds = (EPI == EPI_RFF && TL::LDS < rff_lds) ? rff_lds : TL::LDS;
  hipLaunchKernelGGL((k_gemm_h3<EPI, TL>), dim3(nwg), dim3(TL::NT), lds, stream, a);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}


int check_common(const char* fn, int groups, int rows, int K, const float* A, int lda, const float* W,
                 int ldw) {
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS, "%s: groups=%d", fn, groups);
  AMX_CHECK_ARG(rows >= 0 && rows % AMX_ROW_TILE == 0, "%s: rows=%d must be a multiple of %d", fn, rows,
                AMX_ROW_TILE);
  AMX_CHECK_ARG(K > 0 && K % BK == 0, "%s: K=%d must be a positive multiple of %d", fn, K, BK);
  AMX_CHECK_ARG(A && W, "%s: null operand", fn);
  AMX_CHECK_ARG(amx::aligned16(A) && amx::aligned16(W), "%s: operands must be 16-byte aligned", fn);
  AMX_CHECK_ARG(lda >= K && lda % 4 == 0, "%s: lda=%d (K=%d) must be >= K and a multiple of 4", fn, lda, K);
  AMX_CHECK_ARG(ldw >= K && ldw % 4 == 0, "%s: ldw=%d (K=%d) must be >= K and a multiple of 4", fn, ldw, K);
  return AMX_OK;
}

int check_x6(const char* fn, int groups, int rows, int K, const float* A, int lda, const uint16_t* W3,
             long long strideW3) {
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS, "%s: groups=%d", fn, groups);
  AMX_CHECK_ARG(rows >= 0 && rows % AMX_ROW_TILE == 0, "%s: rows=%d must be a multiple of %d", fn, rows,
                AMX_ROW_TILE);
  AMX_CHECK_ARG(K > 0 && K % XBK == 0, "%s: K=%d must be a positive multiple of %d", fn, K, XBK);
  AMX_CHECK_ARG(A && W3 && amx::aligned16(A) && amx::aligned16(W3), "%s: null/unaligned operand", fn);
  AMX_CHECK_ARG(lda >= K && lda % 4 == 0, "%s: lda=%d (K=%d) must be >= K and a multiple of 4", fn, lda, K);
  AMX_CHECK_ARG(strideW3 % 8 == 0, "%s: strideW3=%lld must be a multiple of 8", fn, strideW3);
  return AMX_OK;
}

int check_h3(const char* fn, int groups, int rows, int K, const float* A, int lda, const uint16_t* W2,
             long long strideW2, const int* w_exp, const int* row_exp, int rexp_slots, int k_shared = 0) {
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS, "%s: groups=%d", fn, groups);
  AMX_CHECK_ARG(rows >= 0 && rows % AMX_ROW_TILE == 0, "%s: rows=%d must be a multiple of %d", fn, rows,
                AMX_ROW_TILE);
  AMX_CHECK_ARG(K > 0 && K % XBK == 0, "%s: K=%d must be a positive multiple of %d", fn, K, XBK);
  AMX_CHECK_ARG(A && W2 && amx::aligned16(A) && amx::aligned16(W2), "%s: null/unaligned operand", fn);
  AMX_CHECK_ARG(lda >= K && lda % 4 == 0, "%s: lda=%d (K=%d) must be >= K and a multiple of 4", fn, lda, K);
  AMX_CHECK_ARG(strideW2 % 8 == 0, "%s: strideW2=%lld must be a multiple of 8", fn, strideW2);
  AMX_CHECK_ARG(w_exp && row_exp && rexp_slots >= 1, "%s: null exponents or rexp_slots=%d", fn, rexp_slots);
  AMX_CHECK_ARG(k_shared >= 0 && k_shared <= K && k_shared % 32 == 0,
                "%s: k_shared=%d must be a multiple of 32 in [0, K=%d]", fn, k_shared, K);
  return AMX_OK;
}

}  // namespace

// ---- f32 MFMA entry points ------------------------------------------------------------------
extern "C" int amx_gemm_bias_act(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                                 long long strideA, const float* W, int ldw, long long strideW,
                                 const float* bias, long long strideBias, float* C, int ldc, long long strideC,
                                 int col_off, int act, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_gemm_bias_act: null ctx");
  int rc = check_common("amx_gemm_bias_act", groups, rows, K, A, lda, W, ldw);
  if (rc) return rc;
  AMX_CHECK_ARG(N > 0 && N % 128 == 0, "amx_gemm_bias_act: N=%d must be a multiple of 128", N);
  AMX_CHECK_ARG(bias && C, "amx_gemm_bias_act: null bias/C");
  AMX_CHECK_ARG(col_off >= 0 && col_off + N <= ldc, "amx_gemm_bias_act: col_off=%d N=%d ldc=%d", col_off, N, ldc);
  AMX_CHECK_ARG(act == AMX_ACT_NONE || act == AMX_ACT_RELU, "amx_gemm_bias_act: act=%d", act);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W = W; a.strideW = strideW; a.ldw = ldw;
  a.bias = bias; a.strideBias = strideBias;
  a.C = C; a.strideC = strideC; a.ldc = ldc; a.col_off = col_off;
  a.rows = rows; a.N = N; a.K = K; a.act = act; a.groups = groups;
  // 128x128, 4 waves of 64x64, two WGs per CU: the main loop keeps the MFMA pipe busy 93-95%
  // of cycles and is then power-limited
  return launch_nt<EPI_BIAS_ACT, T128>(a, (hipStream_t)stream);
}

extern "C" int amx_gemm_out_unnorm(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A,
                                   int lda, long long strideA, const float* W, int ldw, long long strideW,
                                   const float* bias, long long strideBias, float* preds, int ldp,
                                   long long strideP, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "amx_gemm_out_unnorm: context has no normalizers");
  int rc = check_common("amx_gemm_out_unnorm", groups, rows, K, A, lda, W, ldw);
  if (rc) return rc;
  AMX_CHECK_ARG(n_valid == ctx->S, "amx_gemm_out_unnorm: n_valid=%d must equal S=%d", n_valid, ctx->S);
  AMX_CHECK_ARG(bias && preds && ldp >= n_valid, "amx_gemm_out_unnorm: null bias/preds or ldp=%d", ldp);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W = W; a.strideW = strideW; a.ldw = ldw;
  a.bias = bias; a.strideBias = strideBias;
  a.C = preds; a.strideC = strideP; a.ldc = ldp;
  a.rows = rows; a.K = K; a.groups = groups;
  a.n_valid = n_valid;
  const int S = ctx->S, Ad = ctx->A;
  a.shift = ctx->d_norm + 2 * S + 2 * Ad;  // mu_d
  a.scale = ctx->d_norm + 3 * S + 2 * Ad;  // sd_d
  const int n32 = amx::round_up(a.n_valid, 32);
  if (n32 > 128 && n32 <= 224) {  // one 224-wide tile instead of two 128s
    a.N = 224;
    return launch_nt<EPI_UNNORM, T128x224>(a, (hipStream_t)stream);
  }
  a.N = amx::round_up(a.n_valid, 128);
  return launch_nt<EPI_UNNORM, T128>(a, (hipStream_t)stream);
}

extern "C" int amx_rff_features(amx_ctx* ctx, int rows, int n_valid, int F, int K, const float* x, int ldx,
                                const float* W, int ldw, const float* b, float scale, float* phi, int ldphi,
                                double* col_partials, const uint8_t* row_mask, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_rff_features: null ctx");
  int rc = check_common("amx_rff_features", 1, rows, K, x, ldx, W, ldw);
  if (rc) return rc;
  AMX_CHECK_ARG(F > 0 && F % 128 == 0, "amx_rff_features: F=%d must be a multiple of 128", F);
  AMX_CHECK_ARG(b && phi && col_partials && ldphi >= F, "amx_rff_features: null b/phi/partials or ldphi");
  AMX_CHECK_ARG(n_valid >= 0 && n_valid <= rows, "amx_rff_features: n_valid=%d rows=%d", n_valid, rows);
  GemmArgs a = {};
  a.A = x; a.lda = ldx;
  a.W = W; a.ldw = ldw;
  a.bias = b;
  a.C = phi; a.ldc = ldphi;
  a.rows = rows; a.N = F; a.K = K; a.groups = 1;
  a.n_valid = n_valid; a.rff_scale = scale; a.col_partials = col_partials; a.row_mask = row_mask;
  return launch_nt<EPI_RFF, T128>(a, (hipStream_t)stream);
}

// ---- bf16x6 entry points ----------------------------------------------------------------
extern "C" int amx_split_bf16x3(amx_ctx* ctx, int groups, int rows, int K, const float* W, int ldw,
                                long long strideW, uint16_t* W3, long long strideW3, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_split_bf16x3: null ctx");
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS && rows > 0, "amx_split_bf16x3: groups=%d rows=%d", groups,
                rows);
  AMX_CHECK_ARG(K > 0 && K % XBK == 0, "amx_split_bf16x3: K=%d must be a positive multiple of %d", K, XBK);
  AMX_CHECK_ARG(W && W3 && amx::aligned16(W) && amx::aligned16(W3), "amx_split_bf16x3: null/unaligned operand");
  AMX_CHECK_ARG(ldw >= K && ldw % 4 == 0 && strideW3 >= 3LL * K * rows && strideW3 % 8 == 0,
                "amx_split_bf16x3: ldw=%d strideW3=%lld (K=%d rows=%d)", ldw, strideW3, K, rows);
  const long long n = (long long)rows * (K / 4);
  hipLaunchKernelGGL(k_split_bf16x3, dim3((unsigned)((n + 255) / 256), groups), dim3(256), 0, (hipStream_t)stream, W,
                     ldw, strideW, rows, K, W3, strideW3);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_gemm_bias_act_x6(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                                    long long strideA, const uint16_t* W3, long long strideW3, const float* bias,
                                    long long strideBias, float* C, int ldc, long long strideC, int col_off, int act,
                                    void* stream) {
  AMX_CHECK_ARG(ctx, "amx_gemm_bias_act_x6: null ctx");
  int rc = check_x6("amx_gemm_bias_act_x6", groups, rows, K, A, lda, W3, strideW3);
  if (rc) return rc;
  AMX_CHECK_ARG(N > 0 && N % 128 == 0, "amx_gemm_bias_act_x6: N=%d must be a multiple of 128", N);
  AMX_CHECK_ARG(strideW3 >= 3LL * K * N || groups == 1, "amx_gemm_bias_act_x6: strideW3=%lld < 3*K*N", strideW3);
  AMX_CHECK_ARG(bias && C, "amx_gemm_bias_act_x6: null bias/C");
  AMX_CHECK_ARG(col_off >= 0 && col_off + N <= ldc, "amx_gemm_bias_act_x6: col_off=%d N=%d ldc=%d", col_off, N, ldc);
  AMX_CHECK_ARG(act == AMX_ACT_NONE || act == AMX_ACT_RELU, "amx_gemm_bias_act_x6: act=%d", act);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W3 = W3; a.strideW3 = strideW3;
  a.bias = bias; a.strideBias = strideBias;
  a.C = C; a.strideC = strideC; a.ldc = ldc; a.col_off = col_off;
  a.rows = rows; a.N = N; a.K = K; a.act = act; a.groups = groups;
  const hipStream_t s = (hipStream_t)stream;
  // the 256x256 tile halves the operand bytes staged per MFMA against 128x128 (10-14% per
  // hidden layer) when its grid still fills the chip; otherwise 128x128 (2 WGs per CU)
  if (rows % 256 == 0 && N % 256 == 0 &&
      (long long)(rows / 256) * (N / 256) * groups >= resident_wgs(ctx, X256::LDS, X256::NT, 2))
    return launch_x6<EPI_BIAS_ACT, X256>(a, s);
  return launch_x6<EPI_BIAS_ACT, X128>(a, s);
}

extern "C" int amx_gemm_out_unnorm_x6(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A,
                                      int lda, long long strideA, const uint16_t* W3, long long strideW3,
                                      const float* bias, long long strideBias, float* preds, int ldp,
                                      long long strideP, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "amx_gemm_out_unnorm_x6: context has no normalizers");
  int rc = check_x6("amx_gemm_out_unnorm_x6", groups, rows, K, A, lda, W3, strideW3);
  if (rc) return rc;
  AMX_CHECK_ARG(n_valid == ctx->S, "amx_gemm_out_unnorm_x6: n_valid=%d must equal S=%d", n_valid, ctx->S);
  AMX_CHECK_ARG(bias && preds && ldp >= n_valid, "amx_gemm_out_unnorm_x6: null bias/preds or ldp=%d", ldp);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W3 = W3; a.strideW3 = strideW3;
  a.bias = bias; a.strideBias = strideBias;
  a.C = preds; a.strideC = strideP; a.ldc = ldp;
  a.rows = rows; a.K = K; a.groups = groups;
  a.n_valid = n_valid;
  const int S = ctx->S, Ad = ctx->A;
  a.shift = ctx->d_norm + 2 * S + 2 * Ad;  // mu_d
  a.scale = ctx->d_norm + 3 * S + 2 * Ad;  // sd_d
  // weight rows are padded to round_up(S, 128) (amx_layout n_out_pad)
  const int n32 = amx::round_up(n_valid, 32);
  if (n32 > 128 && n32 <= 224) {
    a.N = 224;
    AMX_CHECK_ARG(strideW3 >= 3LL * K * 224 || groups == 1, "amx_gemm_out_unnorm_x6: strideW3=%lld", strideW3);
    return launch_x6<EPI_UNNORM, X128x224>(a, (hipStream_t)stream);
  }
  a.N = amx::round_up(n_valid, 128);
  AMX_CHECK_ARG(strideW3 >= 3LL * K * a.N || groups == 1, "amx_gemm_out_unnorm_x6: strideW3=%lld", strideW3);
  return launch_x6<EPI_UNNORM, X128>(a, (hipStream_t)stream);
}

extern "C" int amx_rff_features_x6(amx_ctx* ctx, int rows, int n_valid, int F, int K, const float* x, int ldx,
                                   const uint16_t* W3, const float* b, float scale, float* phi, int ldphi,
                                   double* col_partials, const uint8_t* row_mask, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_rff_features_x6: null ctx");
  int rc = check_x6("amx_rff_features_x6", 1, rows, K, x, ldx, W3, 0);
  if (rc) return rc;
  AMX_CHECK_ARG(F > 0 && F % 128 == 0, "amx_rff_features_x6: F=%d must be a multiple of 128", F);
  AMX_CHECK_ARG(b && phi && col_partials && ldphi >= F, "amx_rff_features_x6: null b/phi/partials or ldphi");
  AMX_CHECK_ARG(n_valid >= 0 && n_valid <= rows, "amx_rff_features_x6: n_valid=%d rows=%d", n_valid, rows);
  GemmArgs a = {};
  a.A = x; a.lda = ldx;
  a.W3 = W3;
  a.bias = b;
  a.C = phi; a.ldc = ldphi;
  a.rows = rows; a.N = F; a.K = K; a.groups = 1;
  a.n_valid = n_valid; a.rff_scale = scale; a.col_partials = col_partials; a.row_mask = row_mask;
  return launch_x6<EPI_RFF, X128>(a, (hipStream_t)stream);
}

// ---- f16x3 entry points -------------------------------------------------------------------
extern "C" int amx_split_f16x2(amx_ctx* ctx, int groups, int rows, int K, const float* W, int ldw, long long strideW,
                               uint16_t* W2, long long strideW2, int* w_exp, long long strideWexp, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_split_f16x2: null ctx");
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS && rows > 0, "amx_split_f16x2: groups=%d rows=%d", groups,
                rows);
  AMX_CHECK_ARG(K > 0 && K % XBK == 0, "amx_split_f16x2: K=%d must be a positive multiple of %d", K, XBK);
  AMX_CHECK_ARG(W && W2 && w_exp && amx::aligned16(W) && amx::aligned16(W2), "amx_split_f16x2: null/unaligned operand");
  AMX_CHECK_ARG(ldw >= K && ldw % 4 == 0 && strideW2 >= 2LL * K * rows && strideW2 % 8 == 0 && strideWexp >= rows,
                "amx_split_f16x2: ldw=%d strideW2=%lld strideWexp=%lld (K=%d rows=%d)", ldw, strideW2, strideWexp, K,
                rows);
  hipLaunchKernelGGL(k_split_f16x2, dim3((unsigned)((rows + 3) / 4), groups), dim3(256), 0, (hipStream_t)stream, W,
                     ldw, strideW, rows, K, W2, strideW2, w_exp, strideWexp);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_row_exponents(amx_ctx* ctx, int groups, int rows, int K, const float* A, int lda, long long strideA,
                                 int* row_exp, long long strideRexp, int n_slots, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_row_exponents: null ctx");
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS && rows >= 0, "amx_row_exponents: groups=%d rows=%d", groups,
                rows);
  AMX_CHECK_ARG(A && row_exp && K > 0 && lda >= K, "amx_row_exponents: null operand or K=%d lda=%d", K, lda);
  AMX_CHECK_ARG(n_slots >= 1 && n_slots <= 64 && strideRexp >= (long long)n_slots * rows,
                "amx_row_exponents: n_slots=%d strideRexp=%lld rows=%d", n_slots, strideRexp, rows);
  if (rows == 0) return AMX_OK;
  hipLaunchKernelGGL(k_row_exp, dim3((unsigned)((rows + 3) / 4), groups), dim3(256), 0, (hipStream_t)stream, A, lda,
                     strideA, rows, K, row_exp, strideRexp, n_slots);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

// Few rows (128 x 256 hidden tiles would fill less than half the CUs: rows x groups < 8192 at
// N = 512; the reference-semantics sampler's 128-640 rows per member): bm x bn tiles (HS64 /
// HS32), each tile's K range cut into ks = clamp(round(K/32 / 7), 1, 8) contiguous segments of
// about seven K-tiles, one workgroup per segment (k_gemm_h3's stream-K with G = tiles x ks
// workgroups: workgroup v runs units [v U / G, (v + 1) U / G) = segment v % ks of tile v / ks),
// the segments combined in K order by the tile's last arriver (split_combine).  ks depends on K
// alone, so a row's result does not depend on how many rows the launch has (a rank's lanes
// equal the same lanes of one process, bit for bit).  Returns the tile count (0: shape not
// covered), *nwg = G and *ksplit = ks.  (Rounds 3-6 used 128 x 256 tiles split at most 6 ways
// here: 33.7 us per hidden layer at the sampler's 640 lanes, profiles/r06q_paths_trace_summary.txt
// -- each workgroup ran a 10-K-tile chain and wrote a 128 KB partial tile.)
#ifndef SMALL_KT
#define SMALL_KT 7     // K-tiles per segment (target)
#endif
#ifndef SMALL_KSMAX
#define SMALL_KSMAX 8  // segments per tile at most
#endif
static int small_plan(const amx_ctx* ctx, int groups, int rows, int N, int K, int bn, int* nwg, int* ksplit) {
  (void)ctx;
  if (rows <= 0 || rows % 128 != 0 || N % bn != 0 || K % 32 != 0 || groups < 1) return 0;
  const int tiles = rows / 128 * (N / bn) * groups;
  const int nk = K / 32;
  int ks = (nk + SMALL_KT / 2) / SMALL_KT;
  ks = ks < 1 ? 1 : (ks > SMALL_KSMAX ? SMALL_KSMAX : ks);
  if (nwg) *nwg = tiles * ks;
  if (ksplit) *ksplit = ks;
  return tiles;
}

// the hidden layers' shapes that take the small-row tiles
static bool small_hidden(const amx_ctx* ctx, int groups, int rows, int N) {
  return N % 256 == 0 && rows % 128 == 0 && 2LL * (rows / 128) * (N / 256) * groups < ctx->n_cus;
}

extern "C" int amx_gemm_bias_act_h3(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                                    long long strideA, const uint16_t* W2, long long strideW2, const int* w_exp,
                                    long long strideWexp, const float* bias, long long strideBias, float* C, int ldc,
                                    long long strideC, int col_off, int act, const int* row_exp,
                                    long long strideRexp, int rexp_slots, int* row_exp_out, int k_shared,
                                    void* stream) {
  AMX_CHECK_ARG(ctx, "amx_gemm_bias_act_h3: null ctx");
  int rc = check_h3("amx_gemm_bias_act_h3", groups, rows, K, A, lda, W2, strideW2, w_exp, row_exp, rexp_slots,
                    k_shared);
  if (rc) return rc;
  AMX_CHECK_ARG(N > 0 && N % 128 == 0, "amx_gemm_bias_act_h3: N=%d must be a multiple of 128", N);
  AMX_CHECK_ARG(strideW2 >= 2LL * K * N || groups == 1, "amx_gemm_bias_act_h3: strideW2=%lld < 2*K*N", strideW2);
  AMX_CHECK_ARG(bias && C, "amx_gemm_bias_act_h3: null bias/C");
  AMX_CHECK_ARG(col_off >= 0 && col_off + N <= ldc, "amx_gemm_bias_act_h3: col_off=%d N=%d ldc=%d", col_off, N, ldc);
  AMX_CHECK_ARG(act == AMX_ACT_NONE || act == AMX_ACT_RELU, "amx_gemm_bias_act_h3: act=%d", act);
  AMX_CHECK_ARG(strideRexp >= (long long)rexp_slots * rows || groups == 1, "amx_gemm_bias_act_h3: strideRexp=%lld",
                strideRexp);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W2 = W2; a.strideW2 = strideW2; a.w_exp = w_exp; a.strideWexp = strideWexp;
  a.bias = bias; a.strideBias = strideBias;
  a.C = C; a.strideC = strideC; a.ldc = ldc; a.col_off = col_off;
  a.rows = rows; a.N = N; a.K = K; a.act = act; a.groups = groups;
  a.row_exp = row_exp; a.strideRexp = strideRexp; a.rexp_slots = rexp_slots; a.row_exp_out = row_exp_out;
  a.k_shared = k_shared;
  if (ctx->gemm_timer && rexp_slots == 1) { a.timer = ctx->gemm_timer; a.timer_role = 1; }
  const hipStream_t s = (hipStream_t)stream;
  if (rows % 256 == 0 && N % 256 == 0 && K % 32 == 0 &&
      (long long)(rows / 256) * (N / 256) * groups >= resident_wgs(ctx, H256::LDS, H256::NT, 2))
    return H3_W4 ? launch_h3<EPI_BIAS_ACT, H256w4>(a, s) : launch_h3<EPI_BIAS_ACT, H256>(a, s);
  // one wave of row-block tiles: rows = RB * n_cus / (groups * N/256), RB in {128..224}
  if (N % 256 == 0 && K % 32 == 0) {
    const long long per = (long long)groups * (N / 256);
    if (per > 0 && (long long)ctx->n_cus % per == 0 && rows % (ctx->n_cus / per) == 0) {
      switch (rows / (ctx->n_cus / per)) {
        case 128: return launch_h3<EPI_BIAS_ACT, HRow<4>>(a, s);
        case 160: return launch_h3<EPI_BIAS_ACT, HRow<5>>(a, s);
        case 192: return launch_h3<EPI_BIAS_ACT, HRow<6>>(a, s);
        case 224: return launch_h3<EPI_BIAS_ACT, HRow<7>>(a, s);
        default: break;
      }
    }
  }
  if (small_hidden(ctx, groups, rows, N)) {  // few rows (the sampler's lanes): HS64 tiles, stream-K
    int nwg = 0, ksplit = 0;
    const int tiles = small_plan(ctx, groups, rows, N, K, HS64::BN, &nwg, &ksplit);
    if (tiles > 0 && ctx->split_scratch && ctx->split_cnt && ctx->split_ncnt >= tiles &&
        ctx->split_floats >= (long long)tiles * ksplit * HS64::BM * HS64::BN) {
      a.ksplit = ksplit; a.streamk = nwg; a.split_scratch = ctx->split_scratch; a.split_cnt = ctx->split_cnt;
      return rows == 128 ? launch_h3<EPI_BIAS_ACT, HS64w8>(a, s) : launch_h3<EPI_BIAS_ACT, HS64>(a, s);
    }
  }
  if (K % 32 == 0) return launch_h3<EPI_BIAS_ACT, H128k32>(a, s);
  return launch_h3<EPI_BIAS_ACT, H128>(a, s);
}

// Output-layer tiles (128 x 224, S <= 224) of a stream-K launch for `rows` padded lanes x
// `groups` members when the tiles are fewer than the CUs but at least half as many (4096-7168
// lanes x 4 members: 128-224 tiles): one workgroup per CU, the tiles' K-tiles dealt out evenly,
// so a tile's K range spans at most 3 workgroups (*nwg workgroups, *ksplit slots per tile);
// 0 when the shape does not use it.  Fewer tiles than that take the small-row HS32 tiles
// (small_out).
static int streamk_tiles(const amx_ctx* ctx, int groups, int rows, int* nwg = nullptr, int* ksplit = nullptr,
                         int bm = 128) {
  const int n32 = amx::round_up(ctx->S, 32);
  if (n32 <= 128 || n32 > 224 || rows % bm != 0) return 0;
  const int tiles = rows / bm * groups;
  if (tiles < ctx->n_cus && 2 * tiles >= ctx->n_cus) {
    if (nwg) *nwg = ctx->n_cus;
    if (ksplit) *ksplit = 3;
    return tiles;
  }
  return 0;
}

// the output layer's shapes (S <= 224) that take the small-row tiles: fewer 128 x 224 tiles than
// half the CUs (the sampler's lanes; a one-wave 128 x 224 grid ran the whole K = 2304 chain per
// tile, 71 us at 640 lanes in round 3, then 35 us split at most 6 ways)
static bool small_out(const amx_ctx* ctx, int groups, int rows) {
  const int n32 = amx::round_up(ctx->S, 32);
  return n32 > 128 && n32 <= 224 && rows % 128 == 0 && 2LL * (rows / 128) * groups < ctx->n_cus;
}

extern "C" int amx_gemm_out_unnorm_h3(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A,
                                      int lda, long long strideA, const uint16_t* W2, long long strideW2,
                                      const int* w_exp, long long strideWexp, const float* bias, long long strideBias,
                                      float* preds, int ldp, long long strideP, const int* row_exp,
                                      long long strideRexp, int rexp_slots, int k_shared, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "amx_gemm_out_unnorm_h3: context has no normalizers");
  int rc = check_h3("amx_gemm_out_unnorm_h3", groups, rows, K, A, lda, W2, strideW2, w_exp, row_exp, rexp_slots,
                    k_shared);
  if (rc) return rc;
  AMX_CHECK_ARG(n_valid == ctx->S, "amx_gemm_out_unnorm_h3: n_valid=%d must equal S=%d", n_valid, ctx->S);
  AMX_CHECK_ARG(bias && preds && ldp >= n_valid, "amx_gemm_out_unnorm_h3: null bias/preds or ldp=%d", ldp);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W2 = W2; a.strideW2 = strideW2; a.w_exp = w_exp; a.strideWexp = strideWexp;
  a.bias = bias; a.strideBias = strideBias;
  a.C = preds; a.strideC = strideP; a.ldc = ldp;
  a.rows = rows; a.K = K; a.groups = groups;
  a.n_valid = n_valid;
  a.row_exp = row_exp; a.strideRexp = strideRexp; a.rexp_slots = rexp_slots; a.k_shared = k_shared;
  if (ctx->gemm_timer) { a.timer = ctx->gemm_timer; a.timer_role = 2; }
  const int S = ctx->S, Ad = ctx->A;
  a.shift = ctx->d_norm + 2 * S + 2 * Ad;  // mu_d
  a.scale = ctx->d_norm + 3 * S + 2 * Ad;  // sd_d
  const hipStream_t s = (hipStream_t)stream;
  // weight rows padded to round_up(S, 128) (amx_layout n_out_pad); S <= 224 runs one 224-wide tile
  const int n32 = amx::round_up(n_valid, 32);
  // one wave of row-block tiles RB x (N/2) when rows = RB * n_cus / (2 groups), RB in {128..224}
  const int nrb = (2 * groups > 0 && ctx->n_cus % (2 * groups) == 0) ? ctx->n_cus / (2 * groups) : 0;
  const int rb = (nrb > 0 && rows % nrb == 0) ? rows / nrb : 0;
  const bool row_tiles = K % 32 == 0 && (rb == 128 || rb == 160 || rb == 192 || rb == 224);
  if (n32 > 128 && n32 <= 224) {
    a.N = 224;
    AMX_CHECK_ARG(strideW2 >= 2LL * K * 224 || groups == 1, "amx_gemm_out_unnorm_h3: strideW2=%lld", strideW2);
    if (K % 32 != 0) return launch_h3<EPI_UNNORM, H128x224k16>(a, s);
#if OUT80
    if (rows % 80 == 0 && (long long)groups * (rows / 80) == ctx->n_cus) return launch_h3<EPI_UNNORM, H80x224>(a, s);
#endif
    // lane counts whose 128 x 224 tiles (14 waves) are fewer than the CUs (4096-7168 lanes x 4
    // members: 128-224 tiles): stream-K over one workgroup per CU (each tile's K range in <= 3
    // segments), instead of the row-block tiles' 4-7 waves per workgroup
    int nwg = 0, ksplit = 0;
    if (small_out(ctx, groups, rows)) {  // few rows (the sampler's lanes): HS32 tiles, stream-K
      const int tiles = small_plan(ctx, groups, rows, 224, K, HS32::BN, &nwg, &ksplit);
      if (tiles > 0 && ctx->split_scratch && ctx->split_cnt && ctx->split_ncnt >= tiles &&
          ctx->split_floats >= (long long)tiles * ksplit * HS32::BM * HS32::BN) {
        a.ksplit = ksplit; a.streamk = nwg; a.split_scratch = ctx->split_scratch; a.split_cnt = ctx->split_cnt;
        return rows == 128 ? launch_h3<EPI_UNNORM, HS32w8>(a, s) : launch_h3<EPI_UNNORM, HS32>(a, s);
      }
    }
    const int tiles = streamk_tiles(ctx, groups, rows, &nwg, &ksplit);
    if (tiles > 0 && ctx->split_scratch && ctx->split_cnt && ctx->split_ncnt >= tiles &&
        ctx->split_floats >= (long long)tiles * ksplit * 128 * 224) {
      a.ksplit = ksplit; a.streamk = nwg; a.split_scratch = ctx->split_scratch; a.split_cnt = ctx->split_cnt;
      return launch_h3<EPI_UNNORM, H128x224>(a, s);
    }
    if (row_tiles) {
      switch (rb) {
        case 128: return launch_h3<EPI_UNNORM, HOut<4, 7>>(a, s);
        case 160: return launch_h3<EPI_UNNORM, HOut<5, 7>>(a, s);
        case 192: return launch_h3<EPI_UNNORM, HOut<6, 7>>(a, s);
        default: return launch_h3<EPI_UNNORM, HOut<7, 7>>(a, s);
      }
    }
    return launch_h3<EPI_UNNORM, H128x224>(a, s);
  }
  a.N = amx::round_up(n_valid, 128);
  AMX_CHECK_ARG(strideW2 >= 2LL * K * a.N || groups == 1, "amx_gemm_out_unnorm_h3: strideW2=%lld", strideW2);
  if (K % 32 == 0) {
    if (a.N == 256 && row_tiles) {
      switch (rb) {
        case 128: return launch_h3<EPI_UNNORM, HOut<4, 8>>(a, s);
        case 160: return launch_h3<EPI_UNNORM, HOut<5, 8>>(a, s);
        case 192: return launch_h3<EPI_UNNORM, HOut<6, 8>>(a, s);
        default: return launch_h3<EPI_UNNORM, HOut<7, 8>>(a, s);
      }
    }
    if (a.N % 256 == 0) return launch_h3<EPI_UNNORM, H128x256>(a, s);  // the reference scene's S = 226
    return launch_h3<EPI_UNNORM, H128k32>(a, s);
  }
  return launch_h3<EPI_UNNORM, H128>(a, s);
}

extern "C" int amx_rff_features_h3(amx_ctx* ctx, int rows, int n_valid, int F, int K, const float* x, int ldx,
                                   const uint16_t* W2, const int* w_exp, const int* row_exp, const float* b,
                                   float scale, float* phi, int ldphi, double* col_partials, const uint8_t* row_mask,
                                   void* stream) {
  AMX_CHECK_ARG(ctx, "amx_rff_features_h3: null ctx");
  int rc = check_h3("amx_rff_features_h3", 1, rows, K, x, ldx, W2, 0, w_exp, row_exp, 1);
  if (rc) return rc;
  AMX_CHECK_ARG(F > 0 && F % 128 == 0, "amx_rff_features_h3: F=%d must be a multiple of 128", F);
  AMX_CHECK_ARG(b && phi && col_partials && ldphi >= F, "amx_rff_features_h3: null b/phi/partials or ldphi");
  AMX_CHECK_ARG(n_valid >= 0 && n_valid <= rows, "amx_rff_features_h3: n_valid=%d rows=%d", n_valid, rows);
  GemmArgs a = {};
  a.A = x; a.lda = ldx;
  a.W2 = W2; a.w_exp = w_exp;
  a.row_exp = row_exp; a.rexp_slots = 1;
  a.bias = b;
  a.C = phi; a.ldc = ldphi;
  a.rows = rows; a.N = F; a.K = K; a.groups = 1;
  a.n_valid = n_valid; a.rff_scale = scale; a.col_partials = col_partials; a.row_mask = row_mask;
  if (K % 32 == 0) {
    // 160 x 256 tiles where they fill the CUs in whole rounds (see H160x256r)
    if (rows % 160 == 0 && F % 256 == 0 && ((long long)(rows / 160) * (F / 256)) % ctx->n_cus == 0)
      return launch_h3<EPI_RFF, H160x256r>(a, (hipStream_t)stream);
    // (at 40 960 rows the 128 x 128 tile is faster: 121 vs 145 us under the profiler)
    if ((rows / 128) * (F / 128) < ctx->n_cus && F % 64 == 0) return launch_h3<EPI_RFF, H128x64k32>(a, (hipStream_t)stream);
#if RFF_OCC3
    if ((long long)(rows / 128) * (F / 128) > 2LL * ctx->n_cus) return launch_h3<EPI_RFF, H128rff3>(a, (hipStream_t)stream);
#endif
    return launch_h3<EPI_RFF, H128k32>(a, (hipStream_t)stream);
  }
  return launch_h3<EPI_RFF, H128>(a, (hipStream_t)stream);
}

extern "C" int amx_set_gemm_timer(amx_ctx* ctx, uint64_t* buf) {
  AMX_CHECK_ARG(ctx, "amx_set_gemm_timer: null ctx");
  ctx->gemm_timer = buf;
  return AMX_OK;
}

extern "C" int amx_set_split_workspace(amx_ctx* ctx, float* scratch, long long floats, uint32_t* counters,
                                       int n_counters) {
  AMX_CHECK_ARG(ctx, "amx_set_split_workspace: null ctx");
  AMX_CHECK_ARG((scratch == nullptr) == (counters == nullptr) && floats >= 0 && n_counters >= 0,
                "amx_set_split_workspace: scratch and counters must be given together");
  AMX_CHECK_ARG(scratch == nullptr || amx::aligned16(scratch), "amx_set_split_workspace: scratch must be 16-byte aligned");
  ctx->split_scratch = scratch; ctx->split_floats = scratch ? floats : 0;
  ctx->split_cnt = counters; ctx->split_ncnt = counters ? n_counters : 0;
  return AMX_OK;
}

extern "C" long long amx_split_workspace_floats(const amx_ctx* ctx, int groups, int rows, int* n_counters) {
  if (!ctx || groups < 1 || rows <= 0) return -1;
  long long floats = 0;
  int nc = 0;
  auto need = [&](int tiles, int ksplit, int bm, int bn) {
    if (tiles <= 0) return;
    const long long f = (long long)tiles * ksplit * bm * bn;
    floats = f > floats ? f : floats;
    nc = tiles > nc ? tiles : nc;
  };
  int nwg = 0, ksplit = 0;
  const int ldk = ctx->k0_pad + ctx->L * ctx->H;
  const int to = streamk_tiles(ctx, groups, rows, &nwg, &ksplit);
  need(to, ksplit, 128, 224);
  if (small_out(ctx, groups, rows)) {
    const int t = small_plan(ctx, groups, rows, 224, ldk, HS32::BN, &nwg, &ksplit);
    need(t, ksplit, HS32::BM, HS32::BN);
  }
  if (small_hidden(ctx, groups, rows, ctx->H)) {
    for (int i = 0; i < ctx->L; ++i) {  // every hidden layer's K (segments per tile depend on it)
      const int t = small_plan(ctx, groups, rows, ctx->H, ctx->k0_pad + i * ctx->H, HS64::BN, &nwg, &ksplit);
      need(t, ksplit, HS64::BM, HS64::BN);
    }
  }
  if (n_counters) *n_counters = nc;
  return floats;
}
