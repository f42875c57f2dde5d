// Internal building blocks of the GEMM launches (amx_gemm.hip): vector types, GemmArgs, the
// XCD-aware tile map, and the f16x3 tile family (fp32 as two scaled fp16 limbs, three MFMA
// products).
#pragma once

#include "amx_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
// native vector (HIP's float4 is a wrapper struct: arrays of it were not promoted to registers)
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { EPI_BIAS_ACT = 0, EPI_UNNORM = 1, EPI_RFF = 2 };

struct GemmArgs {
  const float* A; long long strideA; int lda;
  const float* W; long long strideW; int ldw;
  const float* bias; long long strideBias;
  float* C; long long strideC; int ldc; int col_off;
  int rows, N, K;
  int act;                 // EPI_BIAS_ACT: AMX_ACT_*
  int n_valid;             // EPI_UNNORM: valid output columns; EPI_RFF: valid rows
  const float* scale;      // EPI_UNNORM: sd_d
  const float* shift;      // EPI_UNNORM: mu_d
  float rff_scale;         // EPI_RFF: sqrt(2/F)
  double* col_partials;    // EPI_RFF: [rows/128][N]
  const uint8_t* row_mask; // EPI_RFF: nullable
  int tiles_m, tiles_n, groups;
  const uint16_t* W3;      // bf16x6 path: 3-limb weight image [g][N][K/16][3][16] (amx_split_bf16x3)
  long long strideW3;      //   elements between groups; a row is 3*K elements
  // f16x3 path (see the section below)
  const uint16_t* W2;      // 2-limb scaled weight image [g][N][K/16][2][16] (amx_split_f16x2)
  long long strideW2;
  const int* w_exp;        // [g][N] column exponents of W2 (strideWexp between groups)
  long long strideWexp;
  const int* row_exp;      // [g][slots][rows]: row exponents of A's column slices
  long long strideRexp;    //   between groups
  int rexp_slots;          //   slices of A read by this launch (exponent = max over them)
  int* row_exp_out;        // nullable: slot receiving the exponents of this launch's output rows
  int k_shared;            // leading K columns of A read from group 0's rows for every group
                           //   (the ensemble's x0 slice, assembled once; multiple of the tile's BK)
  int ksplit;              // partial-tile slots per tile in split_scratch (stream-K output layer)
  int streamk;             // > 0: stream-K over this many workgroups (LATE M16 UNNORM tiles)
  float* split_scratch;    //   raw partial tiles [tile][slot][MB][NB][NT] f32x4 (amx_set_split_workspace)
  uint32_t* split_cnt;     //   arrivals per tile (zero between launches: the last arriver resets it)
  uint64_t* timer;         // amx_set_gemm_timer buffer (null: off)
  int timer_role;          //   1: first layer of a forward (block 0 stamps the start), 2: output layer
};

// Linear block id -> (group, tile_m, tile_n).  Workgroups are dispatched round-robin over
// the 8 XCDs, so block ids congruent mod 8 share an L2.  We hand each XCD a contiguous
// run of logical tiles (tile_n fastest: consecutive tiles reuse the same A row panel;
// then tile_m: they reuse the same weight panels of one ensemble member).  Bijective for
// any tile count (cdna_hip_programming.md T1).
__device__ inline int xcd_logical(int nwg, int orig) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

__device__ inline void tile_coords(const GemmArgs& a, int logical, int& g, int& tm, int& tn) {
  tn = logical % a.tiles_n;
  const int rest = logical / a.tiles_n;
  tm = rest % a.tiles_m;
  g = rest / a.tiles_m;
}

__device__ inline void map_tile(const GemmArgs& a, int orig, int& g, int& tm, int& tn) {
  tile_coords(a, xcd_logical(a.tiles_m * a.tiles_n * a.groups, orig), g, tm, tn);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ==== f16x3: fp32 as two scaled fp16 limbs, three products ==================================
// x = 2^-s (x0 + x1) with x0 = RN_f16(2^s x) and x1 = RN_f16(2^s x - x0): 11 + 11 significant
// bits, |2^s x - x0 - x1| <= 2^-22 |2^s x| (or, below fp16's normal range, 2^-25 absolute
// against a row maximum scaled to [2^13, 2^14)).  a*b is then a0b0 + a0b1 + a1b0 on the f16
// matrix pipe with fp32 accumulation; the dropped a1b1 <= 2^-22 |ab|.  Over a K-long dot
// product these per-term errors add up like sqrt(K) * 2^-23 while the fp32 accumulation of
// the same sum rounds like K * 2^-24, so for K >= ~64 the result carries the same error as an
// fp32 GEMM (measured against fp64: tools/x6_accuracy.py) -- at 3 MFMA per 32x32x16 block
// instead of bf16x6's 6.
//
// The scales are powers of two, so they factor out of the contraction exactly:
//   * weights: per output column c, exponent E_c with max_k |W[c][k]| < 2^E_c, stored
//     scaled by 2^(14 - E_c) (amx_split_f16x2);
//   * activations: per row r, exponent E_r with max_k |A[r][k]| < 2^E_r, scaled by
//     2^(14 - E_r) while staged into LDS.  E_r = max over the row's column slices
//     (row_exp[g][slot][r]); the dense-concat rows are built slice by slice (x0, h0, h1, ...),
//     so the assembly writes slot 0 and each hidden layer's epilogue atomically max-es the
//     exponents of the slice it writes into its own slot (no slot is read and written by the
//     same launch: deterministic).
//   * epilogue: acc * 2^(E_r + E_c - 28) (one exact v_ldexp), then the fp32 bias etc. exactly
//     as the other paths.
// Exponents are clamped to [-100, 100] (zero rows, inf/NaN rows keep propagating as in fp32).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr int HSC = 14;  // scaled operands stay below 2^14 (fp16 max 65504)

__device__ __forceinline__ int exp_of_bits(uint32_t absbits) {
  // E with v < 2^E for v = |x| (bits of a non-negative float); clamped to [-100, 100]
  int e = (int)(absbits >> 23) - 126;
  e = e < -100 ? -100 : e;
  return e > 100 ? 100 : e;
}

// NSUB 16-k granules per K-tile (BK = 16 NSUB); LDS row = NSUB x [limb0 16 | limb1 16] + 8 pad
// (20 dwords at NSUB 1, 36 at NSUB 2: the 16 rows of a ds_read_b128 lane group land on
// distinct 4-bank slots)
template <int WM_, int WN_, int TM_, int TN_, int OCC_ = 2, int NSUB_ = 1, bool LATE_ = false, bool AMAP_ = true,
          bool M16_ = false, int MB16_ = 0, int NB16_ = 0, bool PIN_ = false, bool EARLY_ = false,
          bool SPLIT_ = false, bool DEEPA_ = false, bool SPREAD_ = false>
struct TileH3 {
  static constexpr bool EARLY = EARLY_ && M16_ && LATE_;  // first fragment reads before the publish
  // SPLIT: the publish of tile t+1 and the loads of t+2 are cut into one piece per m-block and
  // placed behind that block's MFMAs (the guide's split write-after-barrier schedule)
  static constexpr bool SPLIT = SPLIT_ && EARLY;
  // DEEPA (SPLIT): the A operand's loads run two K-tiles ahead of its publish instead of one (two
  // register sets; the loop unrolled by two): the output layer's A panel is streamed from HBM
  // once (N = 224 columns per A row), so its K loop waits on load latency, not on the MFMAs
  static constexpr bool DEEPA = DEEPA_ && SPLIT;
  // SPREAD (SPLIT): the staging pieces dealt evenly over the m-blocks (ceil(pieces / MB) behind
  // each) instead of one per block with the rest behind the last
  static constexpr bool SPREAD = SPREAD_ && SPLIT;
  // PIN: sched_barriers keep each block's fragment reads one MFMA group ahead of their use
  static constexpr bool PIN = PIN_;
  static constexpr int WM = WM_, WN = WN_, TM = TM_, TN = TN_, OCC = OCC_, NSUB = NSUB_, BK = 16 * NSUB_;
  // M16: v_mfma_f32_16x16x32_f16 on 16x16 blocks (BK 32; 4 fp32 accumulators per lane and
  // block) instead of 32x32x16 -- the same cycles per FLOP at lower power per FLOP
  // (MI355X_MICROARCH.md); LDS rows of 40 dwords (conflict-free for its lane->k map and for
  // the plain A staging map), the row exponents live in the stage area (160 KB LDS)
  static constexpr bool M16 = M16_;
  static_assert(!M16 || NSUB == 2, "the 16x16x32 MFMA consumes a 32-deep K-tile");
  // AMAP (BK 32): the 16 lanes of a ds_write_b64 group stage rows r and r+2 (36-dword rows:
  // 72 = 8 mod 32 banks apart, so their 2 x 8 dwords interleave) instead of r and r+1 (2-way
  // bank conflict on every A limb store): 2% per layer (tools/h3_variants.py)
  static constexpr bool AMAP = AMAP_ && !M16_;
  // LATE: barrier -> publish tile t+1 -> issue the loads of t+2 -> compute t (write after
  // the barrier: the LDS writes drain under the MFMAs, the loads get a whole K-tile)
  static constexpr bool LATE = LATE_;
  static constexpr int LD = NSUB * 32 + (M16 ? 16 : 8);       // f16 per LDS row
  static constexpr int NT = WM * WN * 64;
  // M16: MB x NB blocks of 16x16 per wave (default 2TM x 2TN; MB16_/NB16_ override, e.g. 7
  // column blocks = 112 columns); 32x32 form: TM x TN blocks of 32x32
  static constexpr int MB = (M16 && MB16_) ? MB16_ : 2 * TM, NB = (M16 && NB16_) ? NB16_ : 2 * TN;
  static constexpr int WROWS = M16 ? MB * 16 : TM * 32, WCOLS = M16 ? NB * 16 : TN * 32;
  static constexpr int BM = WM * WROWS, BN = WN * WCOLS;
  static constexpr int STAGE = (BM + BN) * LD;                 // f16 of one stage (A + W)
  static constexpr size_t LDS = 2 * STAGE * sizeof(uint16_t) + (M16 ? 0 : BM * sizeof(int));
  static constexpr int SEXP = M16 ? STAGE : 2 * STAGE;         // f16 offset of the row exponents
  static constexpr int CPR = 4 * NSUB;                         // 16-B chunks per row and K-tile (A f32 and W)
  static constexpr int NA = BM * CPR, NW = BN * CPR;
  static constexpr int VA = (NA + NT - 1) / NT, VW = (NW + NT - 1) / NT;
  static_assert(LDS <= 160 * 1024, "LDS");
};

// 4 consecutive k of one row, pre-scaled -> two f16 limbs packed as 4 f16 each
__device__ __forceinline__ void split2(f32x4 x, u32x2& l0, u32x2& l1) {
  const f16x4 h0 = __builtin_convertvector(x, f16x4);
  const u32x2 hb = __builtin_bit_cast(u32x2, h0);
  // r1 = x - h0, exact: one mixed-precision fma per element (h0's f16 half widened inside
  // v_fma_mix_f32) instead of a widening convert and a subtract (hipcc folds an fmaf of a
  // widened half back into the convert + subtract, hence the asm)
  f32x4 r1;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r1[0]) : "v"(hb[0]), "v"(x[0]));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1[1]) : "v"(hb[0]), "v"(x[1]));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r1[2]) : "v"(hb[1]), "v"(x[2]));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1[3]) : "v"(hb[1]), "v"(x[3]));
  const f16x4 h1 = __builtin_convertvector(r1, f16x4);
  l0 = __builtin_bit_cast(u32x2, h0);
  l1 = __builtin_bit_cast(u32x2, h1);
}

// One reduce-scatter step of a max over the 32 lanes li: lanes with bit MASK set keep the upper
// HALF values, their partners the lower; each receives the other half (ds_swizzle bitmask
// mode: and 0x1f, xor MASK within 32-lane groups) and keeps the max.
template <int MASK, int HALF>
__device__ __forceinline__ void rs_step(uint32_t* v, int li) {
  const bool up = (li & MASK) != 0;
#pragma unroll
  for (int i = 0; i < HALF; ++i) {
    const uint32_t keep = up ? v[HALF + i] : v[i];
    const uint32_t send = up ? v[i] : v[HALF + i];
    const uint32_t recv = (uint32_t)__builtin_amdgcn_ds_swizzle((int)send, 0x1f | (MASK << 10));
    v[i] = keep > recv ? keep : recv;
  }
}

// amx_set_gemm_timer: the last workgroup of a forward's output layer adds (now - start) to the
// tick sum (stamps only in a buffer nothing else reads)
__device__ __forceinline__ void gemm_timer_end(const GemmArgs& a) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t nwg = gridDim.x;
    if (atomicAdd(reinterpret_cast<unsigned long long*>(a.timer + 1), 1ull) == nwg - 1) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      atomicAdd(reinterpret_cast<unsigned long long*>(a.timer + 2), (unsigned long long)(now - a.timer[0]));
      atomicAdd(reinterpret_cast<unsigned long long*>(a.timer + 3), 1ull);
      atomicExch(reinterpret_cast<unsigned long long*>(a.timer + 1), 0ull);
    }
  }
}

typedef __attribute__((address_space(1))) uint32_t gu32s;

// Stream-K combine (the output layer at lane counts whose 128 x 224 tiles are fewer than the
// CUs: the tiles' K-tiles are dealt out evenly over one workgroup per CU, so a tile's K range is
// covered by nseg <= 3 consecutive workgroups): every segment stores its raw (scaled)
// accumulators write-through (sc1, 16-B per lane) in its slot, drains, and adds to the tile's
// arrival counter (agent scope); the last arriver acquires, sums the segments in K order --
// P0 + P1 + ... whatever the arrival order, so the result is deterministic -- resets the
// counter and returns true to run the epilogue (cdna_hip_programming.md §5, in-launch split-K:
// one release and one acquire per tile).
template <class TL>
__device__ __forceinline__ bool split_combine(const GemmArgs& a, f32x4 (&acc)[TL::MB][TL::NB], int tile, int seg,
                                              int nseg, int* flag) {
  constexpr int MB = TL::MB, NB = TL::NB, NT = TL::NT;
  const int t = threadIdx.x;
  const long long per_slice = (long long)MB * NB * NT;  // f32x4 per slot
  f32x4* base = reinterpret_cast<f32x4*>(a.split_scratch) + (long long)tile * a.ksplit * per_slice;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7ffffff0, 0x00020000);
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[m][n]), rs,
                                             (int)(((seg * MB + m) * NB + n) * NT + t) * 16, 0, 16 /* sc1 */);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add((gu32s*)(a.split_cnt + tile), 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (uint32_t)(nseg - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store((gu32s*)(a.split_cnt + tile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  if constexpr (TL::NT <= 512 && MB * NB * TL::NT <= 2048) {
    // the small-row tiles (HS64 / HS32, 4 or 8 waves): the loads of four segments in flight
    // per round trip (each a write-through partial in memory, ~1-2 us away), then the sums in K
    // order -- v = P0, v += P1, ... exactly as below
    f32x4 v[MB][NB];
    for (int s0 = 0; s0 < nseg; s0 += 4) {
      f32x4 p[4][MB][NB];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s = s0 + q;
        if (s < nseg && s != seg) {
#pragma unroll
          for (int m = 0; m < MB; ++m)
#pragma unroll
            for (int n = 0; n < NB; ++n)
              p[q][m][n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         rs, (int)(((s * MB + m) * NB + n) * NT + t) * 16, 0, 16));
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s = s0 + q;
        if (s < nseg) {
#pragma unroll
          for (int m = 0; m < MB; ++m)
#pragma unroll
            for (int n = 0; n < NB; ++n) {
              const f32x4 x = s == seg ? acc[m][n] : p[q][m][n];
              v[m][n] = s == 0 ? x : v[m][n] + x;
            }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] = v[m][n];
    return true;
  }
  // per block: v = P0, v += P1, ... (own segment from the accumulators) -- the segments' sum in
  // K order without a second copy of the accumulators (which spilled the 128-accumulator tiles).
  // (Round 4: reading this segment's slot back with the others so every segment's loads are in
  // flight together measured no faster at the N = 8 share, profiles/r04a_share_ab.txt.)
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const f32x4 mine = acc[m][n];
      f32x4 v = mine;
      for (int s = 0; s < nseg; ++s) {
        const f32x4 p = s == seg ? mine
                                 : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                 rs, (int)(((s * MB + m) * NB + n) * NT + t) * 16, 0, 16));
        v = s == 0 ? p : v + p;
      }
      acc[m][n] = v;
    }
  return true;
}

}  // namespace
