// EXPERIMENTAL (built only with AMX_EXPERIMENTAL=1: measured slower than the f32-format forward,
// DESIGN.md section 6 round 4).  The ensemble's dense-connect forward on limb-format activations
// ("lb" = limbs), DeviceEnsemble(act_format="limbs") (milo/milo/dynamics.py:216-233, 422-433: BasicMLP's hidden
// layers write relu(x W^T + b) as a new column slice of the concatenated row, the output layer
// reads the whole row).
//
// Why: the f16x3 GEMM (amx_gemm.hip, h3_tile) keeps the activations in fp32 and every consumer
// workgroup splits its A tiles into two scaled fp16 limbs inside the K loop -- VALU work that
// competes with the MFMA issue in every K-tile, redone by every column tile and every later
// layer (profiles/r03d_gemm_noload.txt).  Here each value is split ONCE, by the
// workgroup that produces it:
//   * row layout (same 4 bytes per element as fp32): granules of 16 columns, each
//     [limb0 16 x f16 | limb1 16 x f16]; value = (limb0 + limb1) * 2^(E - 14);
//   * one exponent E per row and CHUNK: chunk 0 = the x0 slice (written by
//     amx_assemble_input_limbs), chunk c >= 1 = columns [k0 + 128 (c-1), k0 + 128 c) (written by
//     the hidden layer that produces them: E = exponent of the chunk's max |h|, row_exp slot c);
//   * the K loop only copies bytes: A and W arrive by LDS-DMA (global_load_lds_dwordx4) into
//     2 or 3 slots, 128-B rows with XOR-swizzled 16-B chunks (physical = logical ^ ((row>>1)&7),
//     on the DMA's per-lane source address and on the fragment read), no VGPR staging, no split,
//     no ds_write pass;
//   * chunks of one row carry different scales, so the fp32 accumulators are rescaled by an exact
//     power of two when the K loop enters a new chunk (acc *= 2^(E_prev - E_next), once per 4
//     K-tiles, one multiply per accumulator) -- the per-row factors come from an LDS table built
//     in the prologue.  To keep |acc| < 2^100 the effective exponent of a chunk is clamped to at
//     least (largest exponent so far) - 60: a chunk 2^60 below the row's largest is weighted as if
//     it were at that floor, an error far below fp32 rounding of the row's sum (all-zero chunks,
//     e.g. dead ReLU blocks, contribute nothing either way).
// The MFMA operands are swapped against h3_tile (v_mfma_f32_16x16x32_f16(W, A)): a lane's
// accumulator then holds one activation row and 4 consecutive output columns, so the hidden
// epilogue writes 8-byte limb runs and needs one exponent per lane and block.
// Same three limb products per 16x16x32 block and K-tile as h3_tile: (a1,b0), (a0,b1), (a0,b0).
#include "amx_common.h"
#include "amx_h3.h"
#include "amx_hip_experimental.h"

#include <type_traits>

namespace {

constexpr int LB_CHUNK = 128;  // columns per exponent chunk of a hidden slice
constexpr int LB_FAC = 24;     // chunks the per-tile factor table holds (K <= k0 + 23 * 128)
constexpr int LB_GAP = 60;     // largest accumulator up-scale between two chunks (2^60)

// WM x WN waves, each MB x NB blocks of 16 x 16 (rows x output columns); R LDS slots of
// [A: BM rows | W: BN rows] x 128 B (one 32-deep K-tile of both limbs).
// REG: the slots are filled through registers (h3_tile's write-after-barrier split schedule:
// after block m's MFMAs, 16-B chunk m of tile t+1 is written to the other slot and reloaded with
// tile t+2 -- a plain copy, the limbs need no split); DEEPA: the A chunks two K-tiles ahead
// (two register sets).  Otherwise LDS-DMA into the R slots (measured slower: with one or two
// K-tiles in flight per CU the K loop waits on the load latency).
template <int WM_, int WN_, int MB_, int NB_, int R_, bool REG_ = true, bool DEEPA_ = false>
struct TileLB {
  static constexpr int WM = WM_, WN = WN_, MB = MB_, NB = NB_, R = R_;
  static constexpr bool REG = REG_, DEEPA = DEEPA_ && REG_;
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int WROWS = MB * 16, WCOLS = NB * 16;
  static constexpr int BM = WM * WROWS, BN = WN * WCOLS, BK = 32;
  static constexpr int A_BYTES = BM * 128, W_BYTES = BN * 128, SLOT = A_BYTES + W_BYTES;
  static constexpr int PA = A_BYTES / 1024, P = SLOT / 1024;  // 1-KB DMA pieces (8 rows) per K-tile
  static constexpr int PMAX = (P + NW - 1) / NW;               // pieces of the first PFULL waves
  static constexpr int PFULL = P % NW == 0 ? NW : P % NW;
  static constexpr int FAC = R * SLOT;                         // fac[LB_FAC][BM] f32
  static constexpr int EFIN = FAC + LB_FAC * BM * 4;           // efin[BM] int: the output unit
  static constexpr int ENDF = EFIN + BM * 4;                   // endf[BM] f32: segment end factor
  static constexpr size_t LDS = (size_t)ENDF + BM * 4;
  static constexpr int NA = BM * 8, NWC = BN * 8;               // 16-B chunks of a K-tile (REG)
  static constexpr int VA = (NA + NT - 1) / NT, VW = (NWC + NT - 1) / NT;
  static_assert(BM % 8 == 0 && BN % 8 == 0 && (R == 2 || R == 3) && (!REG || R == 2) && LDS <= 160 * 1024,
                "limb tile");
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void glb_void_t;

template <int N>
__device__ __forceinline__ void lb_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// chunk of K-tile kt (chunk 0 = the x0 slice's nk0 K-tiles, then 4 K-tiles per chunk)
__device__ __forceinline__ int lb_chunk(int kt, int nk0) { return kt < nk0 ? 0 : 1 + ((kt - nk0) >> 2); }

template <int EPI, class TL>
__device__ __forceinline__ void lb_tile(const GemmArgs& a, int tile, int kb, int ke, int seg, int nseg) {
  constexpr int MB = TL::MB, NB = TL::NB, NW = TL::NW, BM = TL::BM;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* const lds = reinterpret_cast<char*>(smem);
  float* const fac = reinterpret_cast<float*>(lds + TL::FAC);
  int* const efin = reinterpret_cast<int*>(lds + TL::EFIN);
  float* const endf = reinterpret_cast<float*>(lds + TL::ENDF);
  int g, tm, tn;
  tile_coords(a, tile, g, tm, tn);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int lr = lane & 15, q = lane >> 4;
  const int sw = (lr >> 1) & 7;  // fragment rows start at multiples of 16
  const int nk = a.K / TL::BK, nk0 = a.lb_k0 / TL::BK;

  // DMA pieces of this wave: p = wave + NW i (A pieces p < PA first); lane -> row (lane >> 3) of
  // the piece's 8, physical chunk lane & 7 = logical chunk (lane & 7) ^ ((row >> 1) & 7)
  const long long ldw2 = 2LL * a.K;
  const char* src[TL::REG ? 1 : TL::PMAX];
  if constexpr (!TL::REG) {
    const char* Ab = reinterpret_cast<const char*>(a.A + (long long)g * a.strideA + (long long)tm * BM * a.lda);
    const char* Wb = reinterpret_cast<const char*>(a.W2 + (long long)g * a.strideW2 + (long long)tn * TL::BN * ldw2);
    const int prow = lane >> 3, pch = lane & 7;
#pragma unroll
    for (int i = 0; i < TL::PMAX; ++i) {
      const int p = wave + NW * i;
      const bool isA = p < TL::PA;
      const int r = (isA ? p : p - TL::PA) * 8 + prow;
      const int c = pch ^ ((r >> 1) & 7);
      src[i] = isA ? Ab + (long long)r * a.lda * 4 + 16 * c : Wb + (long long)r * ldw2 * 2 + 16 * c;
    }
  }
  const long long x0_back = (long long)g * a.strideA * 4;  // group g's rows -> group 0's (shared x0)
  const int nks = a.k_shared / TL::BK;
  auto issue = [&](int kt, int slot) {
    if constexpr (TL::REG) return;
    char* base = lds + slot * TL::SLOT + wave * 1024;
    const long long ka = (long long)kt * 128 - (kt < nks ? x0_back : 0), kw = (long long)kt * 128;
#pragma unroll
    for (int i = 0; i < TL::PMAX; ++i) {
      const int p = wave + NW * i;
      if (p < TL::P)
        __builtin_amdgcn_global_load_lds((glb_void_t*)(src[i] + (p < TL::PA ? ka : kw)),
                                         (lds_void_t*)(base + NW * i * 1024), 16, 0, 0);
    }
  };
  const bool full = wave < TL::PFULL;

  // the first K-tile's DMA goes out before the exponent table is built (its ordinary loads make
  // hipcc drain the DMA before their use: one K-tile, once)
  if constexpr (!TL::REG) {
    issue(kb, 0);
    if (TL::R == 3 && kb + 1 < ke) issue(kb + 1, 1);
  }

  // per-row chunk factors: fac[c][r] = 2^(E'(c-1) - E'(c)), E'(c) = max(E(c), max_{c'<c} E'(c') - 60);
  // efin[r] = E'(last chunk of the layer): the unit every segment ends in; endf[r] rescales a
  // stream-K segment that stops early to that unit
  {
    const int nch = lb_chunk(nk - 1, nk0) + 1, cend = lb_chunk(ke - 1, nk0);
    for (int r = t; r < BM; r += TL::NT) {
      const int* re = a.row_exp + (long long)g * a.strideRexp + (long long)tm * BM + r;
      // every chunk's exponent loaded at once (one round trip, not one per chunk)
      int ev[LB_FAC];
#pragma unroll
      for (int c = 0; c < LB_FAC; ++c) ev[c] = c < nch ? re[(long long)c * a.rexp_ld] : 0;
      int ee = ev[0], emax = ee, e_end = ee;
#pragma unroll
      for (int c = 1; c < LB_FAC; ++c) {
        if (c >= nch) break;
        const int ec = ev[c];
        const int en = ec > emax - LB_GAP ? ec : emax - LB_GAP;
        fac[c * BM + r] = __builtin_amdgcn_ldexpf(1.0f, ee - en);
        ee = en;
        emax = emax > en ? emax : en;
        if (c == cend) e_end = en;
      }
      efin[r] = ee;
      endf[r] = __builtin_amdgcn_ldexpf(1.0f, e_end - ee);
    }
  }

  f32x4 acc[MB][NB];
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- register staging (REG): chunk q = t + NT j -> row q >> 3, logical 16-B chunk q & 7, written
  // to the physical chunk (q & 7) ^ ((row >> 1) & 7) of its slot row (the DMA layout)
  constexpr int VA = TL::REG ? TL::VA : 1, VW = TL::REG ? TL::VW : 1;
  // chunk j of a thread sits NT/8 rows below chunk j-1: the same swizzle (NT/16 is a multiple of
  // 8), LDS offset + j NT/8 * 128, global offset + j NT/8 rows (a scalar)
  constexpr int RSTEP = TL::NT / 8;
  static_assert(!TL::REG || RSTEP % 16 == 0, "staging rows step");
  const int r0 = t >> 3, c0s = t & 7;
  const int a_src0 = r0 * a.lda * 4 + 16 * c0s, w_src0 = (int)(r0 * ldw2 * 2) + 16 * c0s;
  const int a_dst0 = r0 * 128 + ((c0s ^ ((r0 >> 1) & 7)) << 4), w_dst0 = TL::A_BYTES + a_dst0;
  const int a_step = RSTEP * a.lda * 4, w_step = (int)(RSTEP * ldw2 * 2);
  auto a_ok = [&](int j) { return TL::NA % TL::NT == 0 || j + 1 < VA || t + TL::NT * j < TL::NA; };
  auto w_ok = [&](int j) { return TL::NWC % TL::NT == 0 || j + 1 < VW || t + TL::NT * j < TL::NWC; };
  u32x4 ra[TL::DEEPA ? 2 : 1][VA], rw[VW];
  __amdgpu_buffer_rsrc_t rsA, rsA0, rsW;
  if constexpr (TL::REG) {
    const float* Ab = a.A + (long long)g * a.strideA + (long long)tm * BM * a.lda;
    const float* Ab0 = a.A + (long long)tm * BM * a.lda;
    const uint16_t* Wb = a.W2 + (long long)g * a.strideW2 + (long long)tn * TL::BN * ldw2;
    rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Ab), 0, 0x7ffffff0, 0x00020000);
    rsA0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Ab0), 0, 0x7ffffff0, 0x00020000);
    rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Wb), 0, 0x7ffffff0, 0x00020000);
  }
  auto gA = [&](int j, int kt) -> u32x4 {
    kt = kt < nk ? kt : nk - 1;  // past the end: re-read the last tile (branch-free)
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(kt < nks ? rsA0 : rsA, a_src0,
                                                                          kt * 128 + j * a_step, 0));
  };
  auto gW = [&](int j, int kt) -> u32x4 {
    kt = kt < nk ? kt : nk - 1;
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsW, w_src0, kt * 128 + j * w_step, 0));
  };
  auto load_a = [&](auto set, int kt) {
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok(j)) ra[decltype(set)::value][j] = gA(j, kt);
  };
  auto load_w = [&](int kt) {
#pragma unroll
    for (int j = 0; j < VW; ++j)
      if (w_ok(j)) rw[j] = gW(j, kt);
  };
  auto publish = [&](int slot, auto set) {
    char* S0 = lds + slot * TL::SLOT;
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok(j)) *reinterpret_cast<u32x4*>(S0 + a_dst0 + j * RSTEP * 128) = ra[decltype(set)::value][j];
#pragma unroll
    for (int j = 0; j < VW; ++j)
      if (w_ok(j)) *reinterpret_cast<u32x4*>(S0 + w_dst0 + j * RSTEP * 128) = rw[j];
  };
  // one staging piece: A chunk qq (or W chunk qq - VA) of the registered tile into `slot`, then the
  // register reloaded with tile kt (A: kt + 1 with DEEPA, two tiles ahead of W)
  auto piece = [&](int qq, int slot, int kt, auto set) {
    char* S0 = lds + slot * TL::SLOT;
    if (qq < VA) {
      if (a_ok(qq)) {
        *reinterpret_cast<u32x4*>(S0 + a_dst0 + qq * RSTEP * 128) = ra[decltype(set)::value][qq];
        ra[decltype(set)::value][qq] = gA(qq, TL::DEEPA ? kt + 1 : kt);
      }
    } else if (qq < VA + VW) {
      const int j = qq - VA;
      if (w_ok(j)) {
        *reinterpret_cast<u32x4*>(S0 + w_dst0 + j * RSTEP * 128) = rw[j];
        rw[j] = gW(j, kt);
      }
    }
  };
  // fragment offsets: k = 8q..8q+7 of limb L = logical chunk 4 (q >> 1) + 2 L + (q & 1)
  const int c0 = ((4 * (q >> 1) + (q & 1)) ^ sw) * 16, c1 = ((4 * (q >> 1) + 2 + (q & 1)) ^ sw) * 16;
  const int a_off = (wm * TL::WROWS + lr) * 128, w_off = TL::A_BYTES + (wn * TL::WCOLS + lr) * 128;
  const int frow = wm * TL::WROWS + lr;  // the lane's accumulator row (block m: + 16 m)
  // compute(tile in `slot`); REG: behind block m's MFMAs, staging piece m writes chunk m of the
  // registered tile into `pslot` and reloads it with tile pkt (set: the A register set)
  auto compute = [&](int slot, bool resc, int chunk, int pslot, int pkt, auto set) {
    const char* S0 = lds + slot * TL::SLOT;
    f16x8 wb[NB][2], ah[2], al[2];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const char* wr = S0 + w_off + n * 16 * 128;
      wb[n][0] = *reinterpret_cast<const f16x8*>(wr + c0);
      wb[n][1] = *reinterpret_cast<const f16x8*>(wr + c1);
    }
    ah[0] = *reinterpret_cast<const f16x8*>(S0 + a_off + c0);
    al[0] = *reinterpret_cast<const f16x8*>(S0 + a_off + c1);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      if (m + 1 < MB) {
        const char* ar = S0 + a_off + (m + 1) * 16 * 128;
        ah[(m + 1) & 1] = *reinterpret_cast<const f16x8*>(ar + c0);
        al[(m + 1) & 1] = *reinterpret_cast<const f16x8*>(ar + c1);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (resc) {  // a new chunk starts at this K-tile: the block's accumulators into its unit
        const float f = fac[chunk * BM + frow + 16 * m];
#pragma unroll
        for (int n = 0; n < NB; ++n) acc[m][n] *= f;
      }
#pragma unroll
      for (int n = 0; n < NB; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb[n][0], al[m & 1], acc[m][n], 0, 0, 0);
#pragma unroll
      for (int n = 0; n < NB; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb[n][1], ah[m & 1], acc[m][n], 0, 0, 0);
#pragma unroll
      for (int n = 0; n < NB; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb[n][0], ah[m & 1], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (TL::REG) {
        piece(m, pslot, pkt, set);
        if (m == MB - 1) {
#pragma unroll
          for (int qq = MB; qq < TL::VA + TL::VW; ++qq) piece(qq, pslot, pkt, set);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  using S0_ = std::integral_constant<int, 0>;
  using S1_ = std::integral_constant<int, 1>;
  if constexpr (TL::REG && TL::DEEPA) {
    // tile x's A in register set (x - kb) & 1, loaded two tiles ahead; W one tile ahead
    load_a(S0_{}, kb);
    load_w(kb);
    publish(0, S0_{});
    load_a(S1_{}, kb + 1);
    load_w(kb + 1);
    load_a(S0_{}, kb + 2);
    auto kstep = [&](int kt, auto par) {  // slot par; pieces publish tile kt+1 from set par ^ 1
      constexpr int P = decltype(par)::value;
      __syncthreads();  // tile kt visible in slot P; slot P ^ 1 (tile kt - 1) fully read
      const int ch = lb_chunk(kt, nk0);
      compute(P, kt > kb && ch != lb_chunk(kt - 1, nk0), ch, P ^ 1, kt + 2, std::integral_constant<int, P ^ 1>{});
    };
    for (int kt = kb; kt < ke; kt += 2) {
      kstep(kt, S0_{});
      if (kt + 1 < ke) kstep(kt + 1, S1_{});
    }
  } else if constexpr (TL::REG) {
    load_a(S0_{}, kb);
    load_w(kb);
    publish(0, S0_{});
    load_a(S0_{}, kb + 1);
    load_w(kb + 1);
    for (int kt = kb; kt < ke; ++kt) {
      const int cur = (kt - kb) & 1;
      __syncthreads();  // tile kt visible in slot cur; slot cur ^ 1 (tile kt - 1) fully read
      const int ch = lb_chunk(kt, nk0);
      compute(cur, kt > kb && ch != lb_chunk(kt - 1, nk0), ch, cur ^ 1, kt + 2, S0_{});
    }
  } else if constexpr (TL::R == 2) {
    for (int kt = kb; kt < ke; ++kt) {
      const int cur = (kt - kb) & 1;
      lb_wait_barrier<0>();  // tile kt landed (every wave's pieces); tile kt-1's slot fully read
      if (kt + 1 < ke) issue(kt + 1, cur ^ 1);
      const int ch = lb_chunk(kt, nk0);
      compute(cur, kt > kb && ch != lb_chunk(kt - 1, nk0), ch, 0, 0, S0_{});
    }
  } else {
    int slot = 0;  // (kt - kb) % 3
    for (int kt = kb; kt < ke; ++kt) {
      if (kt + 1 >= ke) lb_wait_barrier<0>();
      else if (full) lb_wait_barrier<TL::PMAX>();  // tile kt+1's pieces may stay in flight
      else lb_wait_barrier<TL::PMAX - 1>();
      if (kt + 2 < ke) issue(kt + 2, slot == 0 ? 2 : slot - 1);  // the slot tile kt-1 used
      const int ch = lb_chunk(kt, nk0);
      compute(slot, kt > kb && ch != lb_chunk(kt - 1, nk0), ch, 0, 0, S0_{});
      slot = slot == 2 ? 0 : slot + 1;
    }
  }

  if (nseg > 1) {  // stream-K: this segment's partial sums into the layer's final unit, then combine
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const float f = endf[frow + 16 * m];
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[m][n] *= f;
    }
    __syncthreads();  // the slots are free: one int of LDS for the last-arriver flag
    if (!split_combine<TL>(a, acc, tile, seg, nseg, reinterpret_cast<int*>(smem))) return;
  }

  const float* bias = a.bias + (long long)g * a.strideBias;
  const int* wexp = a.w_exp + (long long)g * a.strideWexp;
  float* Cg = a.C + (long long)g * a.strideC;
  const int col0 = tn * TL::BN + wn * TL::WCOLS + 4 * q;  // + 16 n + j
  if constexpr (EPI == EPI_UNNORM) {
    int er[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) er[m] = efin[frow + 16 * m] - 2 * HSC;
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = col0 + 16 * n + j;
        if (col < a.n_valid) {
          const float bv = bias[col], sc = a.scale[col], sh = a.shift[col];
          const int ec = wexp[col];
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            const long long row = (long long)tm * BM + frow + 16 * m;
            const float y = __builtin_amdgcn_ldexpf(acc[m][n][j], er[m] + ec) + bv;
            const float prod = y * sc;  // two roundings, as torch's (y*scale)+mean
            Cg[row * a.ldc + col] = prod + sh;
          }
        }
      }
  } else {  // EPI_BIAS_ACT: relu(x W^T + b) as limbs + the chunk exponents
    static_assert(TL::WCOLS == 64 && TL::WN % 2 == 0, "a 128-column chunk = the columns of waves wn, wn ^ 1");
    uint32_t mx[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int er = efin[frow + 16 * m] - 2 * HSC;
      uint32_t r = 0u;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + col0 + 16 * n);
        const int4 ec = *reinterpret_cast<const int4*>(wexp + col0 + 16 * n);
        const int ecv[4] = {ec.x, ec.y, ec.z, ec.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = __builtin_amdgcn_ldexpf(acc[m][n][j], er + ecv[j]) + bv[j];
          if (a.act == AMX_ACT_RELU) v = (v < 0.f) ? 0.f : v;  // keeps NaN, as torch.relu
          acc[m][n][j] = v;
          const uint32_t b = __float_as_uint(v) & 0x7fffffffu;
          r = r > b ? r : b;
        }
      }
      // max over the row's 64 columns of this wave: the lanes lr, lr + 16, lr + 32, lr + 48
      uint32_t o = (uint32_t)__shfl_xor((int)r, 16);
      r = r > o ? r : o;
      o = (uint32_t)__shfl_xor((int)r, 32);
      mx[m] = r > o ? r : o;
    }
    __syncthreads();  // every wave is done with the slots: [WN][BM] row maxima after the flag word
    uint32_t* smx = reinterpret_cast<uint32_t*>(lds + 16);
    if (q == 0) {
#pragma unroll
      for (int m = 0; m < MB; ++m) smx[wn * BM + frow + 16 * m] = mx[m];
    }
    __syncthreads();
    const int chunk = (tn * TL::BN + wn * TL::WCOLS) / LB_CHUNK;  // chunk of this layer's slice
    int* eout = a.row_exp_out ? a.row_exp_out + (long long)g * a.strideRexp + (long long)chunk * a.rexp_ld : nullptr;
    const int gran = (a.col_off + tn * TL::BN + wn * TL::WCOLS) / 16;  // first granule of the wave's columns
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int rl = frow + 16 * m;
      const uint32_t p = smx[(wn ^ 1) * BM + rl];
      const int E = exp_of_bits(mx[m] > p ? mx[m] : p);
      const long long row = (long long)tm * BM + rl;
      if (eout && (wn & 1) == 0 && q == 0) eout[row] = E;
      float* dst = Cg + row * a.ldc + 16 * gran + 2 * q;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        f32x4 x = acc[m][n];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = __builtin_amdgcn_ldexpf(x[j], HSC - E);
        u32x2 l0, l1;
        split2(x, l0, l1);
        *reinterpret_cast<u32x2*>(dst + 16 * n) = l0;
        *reinterpret_cast<u32x2*>(dst + 16 * n + 8) = l1;
      }
    }
  }
}

template <int EPI, class TL>
__global__ __launch_bounds__(TL::NT, 1) void k_gemm_lb(GemmArgs a) {
  if (a.timer_role == 1 && blockIdx.x == 0 && threadIdx.x == 0) a.timer[0] = __builtin_amdgcn_s_memrealtime();
  const int nk = a.K / TL::BK;
  if (a.streamk) {  // k_gemm_h3's stream-K deal: one workgroup per CU or SPLIT per tile
    const long long U = (long long)a.tiles_m * a.tiles_n * a.groups * nk, G = gridDim.x;
    const int v = xcd_logical((int)G, (int)blockIdx.x);
    long long u = (long long)v * U / G;
    const long long uend = ((long long)v + 1) * U / G;
    while (u < uend) {
      const int tile = (int)(u / nk), kb = (int)(u - (long long)tile * nk);
      const int ke = (uend - u) < (long long)(nk - kb) ? kb + (int)(uend - u) : nk;
      const long long u0 = (long long)tile * nk;
      const int wf = (int)(((u0 + 1) * G - 1) / U), wl = (int)(((u0 + nk) * G - 1) / U);
      lb_tile<EPI, TL>(a, tile, kb, ke, v - wf, wl - wf + 1);
      u += ke - kb;
      __syncthreads();  // LDS reuse by the next segment
    }
  } else {
    lb_tile<EPI, TL>(a, xcd_logical(a.tiles_m * a.tiles_n * a.groups, (int)blockIdx.x), 0, nk, 0, 1);
  }
  if (a.timer_role == 2) gemm_timer_end(a);
}

// hidden tiles: 8 waves (2 x 4) of MB*16 rows x 64 columns, 256 columns per tile, register-staged
template <int MB> using LBHid = TileLB<2, 4, MB, 4, 2>;
// output tiles: 128 rows, BN / 32 waves (2 x BN/32) of 64 rows x 32 columns (h3's 128 x 224 geometry),
// register-staged with A two K-tiles ahead
template <int BN> using LBOut = TileLB<2, BN / 32, 4, 2, 2, true, true>;
// the LDS-DMA forms (amx_set_lb_stage 1; A/B)
template <int MB> using LBHidDma = TileLB<2, 4, MB, 4, 2, false>;
template <int NB> using LBOutDma = TileLB<4, 2, 2, NB, 3, false>;

template <int EPI, class TL>
int launch_lb(GemmArgs& a, hipStream_t stream) {
  a.tiles_m = a.rows / TL::BM;
  a.tiles_n = a.N / TL::BN;
  const int tiles = a.tiles_m * a.tiles_n * a.groups;
  const int nwg = a.streamk ? a.streamk : tiles;
  if (tiles == 0) return AMX_OK;
  hipLaunchKernelGGL((k_gemm_lb<EPI, TL>), dim3(nwg), dim3(TL::NT), TL::LDS, stream, a);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

int check_lb(const char* fn, int groups, int rows, int K, const float* A, int lda, const uint16_t* W2,
             long long strideW2, const int* w_exp, const int* row_exp, long long rexp_ld, int k0, int k_shared) {
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS, "%s: groups=%d", fn, groups);
  AMX_CHECK_ARG(rows >= 0 && rows % AMX_ROW_TILE == 0, "%s: rows=%d must be a multiple of %d", fn, rows,
                AMX_ROW_TILE);
  AMX_CHECK_ARG(k0 > 0 && k0 % 32 == 0 && K >= k0 && (K - k0) % LB_CHUNK == 0,
                "%s: K=%d, k0=%d: k0 must be a positive multiple of 32 and K - k0 a multiple of %d", fn, K, k0,
                LB_CHUNK);
  AMX_CHECK_ARG(1 + (K - k0) / LB_CHUNK <= LB_FAC, "%s: K=%d has more than %d exponent chunks", fn, K, LB_FAC);
  AMX_CHECK_ARG(A && W2 && amx::aligned16(A) && amx::aligned16(W2), "%s: null/unaligned operand", fn);
  AMX_CHECK_ARG(lda >= K && lda % 4 == 0, "%s: lda=%d (K=%d) must be >= K and a multiple of 4", fn, lda, K);
  AMX_CHECK_ARG(strideW2 % 8 == 0, "%s: strideW2=%lld must be a multiple of 8", fn, strideW2);
  AMX_CHECK_ARG(w_exp && row_exp && rexp_ld >= rows, "%s: null exponents or rexp_ld=%lld < rows", fn, rexp_ld);
  AMX_CHECK_ARG(k_shared == 0 || k_shared == k0, "%s: k_shared=%d must be 0 or k0=%d", fn, k_shared, k0);
  return AMX_OK;
}

// stream-K decomposition over a tile grid smaller than the chip (k_gemm_h3's rules): tiles in
// [CUs/2, CUs): one workgroup per CU, <= 3 segments per tile; fewer: SPLIT = min(CUs/tiles, 6)
// workgroups per tile of >= 4 K-tiles each.  0: one workgroup per tile.
int lb_streamk(const amx_ctx* ctx, int tiles, int nk, int* nwg, int* ksplit) {
  if (tiles >= ctx->n_cus || tiles < 1) return 0;
  if (2 * tiles >= ctx->n_cus) {
    *nwg = ctx->n_cus;
    *ksplit = 3;
    return 1;
  }
  int split = ctx->n_cus / tiles;
  split = split > 6 ? 6 : split;
  while (split > 1 && nk / split < 4) --split;
  if (split < 2) return 0;
  *nwg = tiles * split;
  *ksplit = split;
  return 1;
}

bool lb_use_streamk(const amx_ctx* ctx, GemmArgs& a, int tiles, int bm, int bn) {
  int nwg = 0, ksplit = 0;
  if (!lb_streamk(ctx, tiles, a.K / 32, &nwg, &ksplit)) return false;
  if (!ctx->split_scratch || !ctx->split_cnt || ctx->split_ncnt < tiles ||
      ctx->split_floats < (long long)tiles * ksplit * bm * bn)
    return false;
  a.ksplit = ksplit; a.streamk = nwg; a.split_scratch = ctx->split_scratch; a.split_cnt = ctx->split_cnt;
  return true;
}

struct LBHidSel {
  template <int MB> using T = LBHid<MB>;
};
struct LBHidDmaSel {
  template <int MB> using T = LBHidDma<MB>;
};

// the hidden-layer tile choice of amx_gemm_bias_act_lb for a tile family SEL::T<MB>
template <class SEL>
int lb_hidden(const amx_ctx* ctx, GemmArgs& a, int rows, long long per, hipStream_t s) {
  if (per > 0 && ctx->n_cus % per == 0 && (rows * per) % ctx->n_cus == 0) {
    const long long bm = rows * per / ctx->n_cus;
    if (bm % 32 == 0 && rows % bm == 0) {
      switch (bm) {
        case 128: return launch_lb<EPI_BIAS_ACT, typename SEL::template T<4>>(a, s);
        case 160: return launch_lb<EPI_BIAS_ACT, typename SEL::template T<5>>(a, s);
        case 192: return launch_lb<EPI_BIAS_ACT, typename SEL::template T<6>>(a, s);
        case 224: return launch_lb<EPI_BIAS_ACT, typename SEL::template T<7>>(a, s);
        case 256: return launch_lb<EPI_BIAS_ACT, typename SEL::template T<8>>(a, s);
        default: break;
      }
    }
  }
  if (rows % 256 == 0 && rows / 256 * per >= ctx->n_cus)
    return launch_lb<EPI_BIAS_ACT, typename SEL::template T<8>>(a, s);
  const int t128 = (int)(rows / 128 * per);
  if (2 * t128 < ctx->n_cus) lb_use_streamk(ctx, a, t128, 128, 256);
  return launch_lb<EPI_BIAS_ACT, typename SEL::template T<4>>(a, s);
}

// ---- x0 as limbs --------------------------------------------------------------------------
// x0 = [(s - mu_s)/sd_s, (a - mu_a)/sd_a, 0...] (dynamics.py:225-227), one wave per lane row,
// 4 consecutive columns per lane: the row's max |x0| gives E (row_exp slot 0, every model), then
// the values are split as limbs with scale 2^(14 - E), into model 0's rows (stride_m 0: every
// model's GEMMs read that one copy) or every model's.
template <typename T>
__global__ __launch_bounds__(256) void k_assemble_limbs(const T* __restrict__ ob, const T* __restrict__ act,
                                                        const float* __restrict__ norm, float* __restrict__ buf,
                                                        long long stride_m, int ldk, int S, int A, int M, int k0,
                                                        int B, int* __restrict__ row_exp, long long stride_rexp) {
  constexpr int MAXP = 4;  // k0 <= 1024
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* mu_s = norm;
  const float* sd_s = norm + S;
  const float* mu_a = norm + 2 * S;
  const float* sd_a = norm + 2 * S + A;
  f32x4 x[MAXP];
  uint32_t mx = 0;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 256 * p + 4 * lane + i;
      float v = 0.f;
      if (j < S) {
        v = ((float)ob[(long long)b * S + j] - mu_s[j]) / sd_s[j];
      } else if (j < S + A) {
        const int k = j - S;
        v = ((float)act[(long long)b * A + k] - mu_a[k]) / sd_a[k];
      }
      x[p][i] = v;
      const uint32_t bits = __float_as_uint(v) & 0x7fffffffu;
      mx = mx > bits ? mx : bits;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)mx, off);
    mx = mx > o ? mx : o;
  }
  const int E = exp_of_bits(mx);
  const int copies = stride_m == 0 ? 1 : M;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int j = 256 * p + 4 * lane;
    if (j >= k0) break;
    f32x4 v = x[p];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_ldexpf(v[i], HSC - E);
    u32x2 l0, l1;
    split2(v, l0, l1);
    const long long off = (long long)b * ldk + 16 * (j / 16) + 2 * ((j % 16) / 4);
    for (int m = 0; m < copies; ++m) {
      *reinterpret_cast<u32x2*>(buf + m * stride_m + off) = l0;
      *reinterpret_cast<u32x2*>(buf + m * stride_m + off + 8) = l1;
    }
  }
  if (lane == 0)
    for (int m = 0; m < M; ++m) row_exp[m * stride_rexp + b] = E;
}

}  // namespace

extern "C" int amx_assemble_input_limbs(amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                                        long long stride_m, int ldk, int B, int* row_exp, long long strideRexp,
                                        void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "amx_assemble_input_limbs: context has no normalizers");
  AMX_CHECK_ARG(ob && act && act_buf && row_exp && B >= 0, "amx_assemble_input_limbs: null pointer or B=%d", B);
  AMX_CHECK_ARG(in_dtype == AMX_IN_F64 || in_dtype == AMX_IN_F32, "amx_assemble_input_limbs: in_dtype=%d", in_dtype);
  AMX_CHECK_ARG(ctx->k0_pad <= 1024 && ctx->k0_pad % 16 == 0 && ldk >= ctx->k0_pad && ldk % 4 == 0 &&
                    amx::aligned16(act_buf),
                "amx_assemble_input_limbs: k0=%d ldk=%d (k0 <= 1024, 16-B aligned rows)", ctx->k0_pad, ldk);
  AMX_CHECK_ARG(ctx->M == 1 || strideRexp >= B, "amx_assemble_input_limbs: strideRexp=%lld", strideRexp);
  if (B == 0) return AMX_OK;
  const dim3 grid((unsigned)((B + 3) / 4));
  const hipStream_t s = (hipStream_t)stream;
  if (in_dtype == AMX_IN_F64)
    hipLaunchKernelGGL(k_assemble_limbs<double>, grid, dim3(256), 0, s, (const double*)ob, (const double*)act,
                       ctx->d_norm, act_buf, stride_m, ldk, ctx->S, ctx->A, ctx->M, ctx->k0_pad, B, row_exp, strideRexp);
  else
    hipLaunchKernelGGL(k_assemble_limbs<float>, grid, dim3(256), 0, s, (const float*)ob, (const float*)act,
                       ctx->d_norm, act_buf, stride_m, ldk, ctx->S, ctx->A, ctx->M, ctx->k0_pad, B, row_exp, strideRexp);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_gemm_bias_act_lb(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                                    long long strideA, const uint16_t* W2, long long strideW2, const int* w_exp,
                                    long long strideWexp, const float* bias, long long strideBias, float* C, int ldc,
                                    long long strideC, int col_off, int act, const int* row_exp, long long strideRexp,
                                    long long rexp_ld, int* row_exp_out, int k0, int k_shared, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_gemm_bias_act_lb: null ctx");
  int rc = check_lb("amx_gemm_bias_act_lb", groups, rows, K, A, lda, W2, strideW2, w_exp, row_exp, rexp_ld, k0,
                    k_shared);
  if (rc) return rc;
  AMX_CHECK_ARG(N > 0 && N % 256 == 0, "amx_gemm_bias_act_lb: N=%d must be a multiple of 256", N);
  AMX_CHECK_ARG(strideW2 >= 2LL * K * N || groups == 1, "amx_gemm_bias_act_lb: strideW2=%lld < 2*K*N", strideW2);
  AMX_CHECK_ARG(bias && C && amx::aligned16(bias) && amx::aligned16(w_exp) && strideBias % 4 == 0 &&
                    strideWexp % 4 == 0,
                "amx_gemm_bias_act_lb: null/unaligned bias, w_exp or their group strides");
  AMX_CHECK_ARG(col_off >= k0 && (col_off - k0) % LB_CHUNK == 0 && col_off + N <= ldc && ldc % 4 == 0,
                "amx_gemm_bias_act_lb: col_off=%d N=%d ldc=%d (k0=%d)", col_off, N, ldc, k0);
  AMX_CHECK_ARG(act == AMX_ACT_NONE || act == AMX_ACT_RELU, "amx_gemm_bias_act_lb: act=%d", act);
  AMX_CHECK_ARG(row_exp_out, "amx_gemm_bias_act_lb: row_exp_out is required (the output chunks' exponents)");
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W2 = W2; a.strideW2 = strideW2; a.w_exp = w_exp; a.strideWexp = strideWexp;
  a.bias = bias; a.strideBias = strideBias;
  a.C = C; a.strideC = strideC; a.ldc = ldc; a.col_off = col_off;
  a.rows = rows; a.N = N; a.K = K; a.act = act; a.groups = groups;
  a.row_exp = row_exp; a.strideRexp = strideRexp; a.rexp_ld = rexp_ld; a.row_exp_out = row_exp_out;
  a.lb_k0 = k0; a.k_shared = k_shared;
  if (ctx->gemm_timer && K == k0) { a.timer = ctx->gemm_timer; a.timer_role = 1; }
  const hipStream_t s = (hipStream_t)stream;
  // one wave of row-block tiles (BM rows = 32 MB) when rows x N/256 x groups / BM fills the CUs
  // exactly, else 256-row tiles over several waves, else stream-K 128-row tiles, else 128-row tiles
  const long long per = (long long)groups * (N / 256);
  // one wave of row-block tiles (BM rows = 32 MB) when rows x N/256 x groups / BM fills the CUs
  // exactly, else 256-row tiles over several waves, else stream-K 128-row tiles (few tiles only:
  // at [CUs/2, CUs) tiles the partial tiles cost more than the idle CUs), else
  // 128-row tiles
  if (ctx->lb_stage == 1) return lb_hidden<LBHidDmaSel>(ctx, a, rows, per, s);
  return lb_hidden<LBHidSel>(ctx, a, rows, per, s);
}

extern "C" int amx_gemm_out_unnorm_lb(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A,
                                      int lda, long long strideA, const uint16_t* W2, long long strideW2,
                                      const int* w_exp, long long strideWexp, const float* bias, long long strideBias,
                                      float* preds, int ldp, long long strideP, const int* row_exp,
                                      long long strideRexp, long long rexp_ld, int k0, int k_shared, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "amx_gemm_out_unnorm_lb: context has no normalizers");
  int rc = check_lb("amx_gemm_out_unnorm_lb", groups, rows, K, A, lda, W2, strideW2, w_exp, row_exp, rexp_ld, k0,
                    k_shared);
  if (rc) return rc;
  AMX_CHECK_ARG(n_valid == ctx->S, "amx_gemm_out_unnorm_lb: n_valid=%d must equal S=%d", n_valid, ctx->S);
  AMX_CHECK_ARG(bias && preds && ldp >= n_valid, "amx_gemm_out_unnorm_lb: null bias/preds or ldp=%d", ldp);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W2 = W2; a.strideW2 = strideW2; a.w_exp = w_exp; a.strideWexp = strideWexp;
  a.bias = bias; a.strideBias = strideBias;
  a.C = preds; a.strideC = strideP; a.ldc = ldp;
  a.rows = rows; a.K = K; a.groups = groups;
  a.n_valid = n_valid;
  a.row_exp = row_exp; a.strideRexp = strideRexp; a.rexp_ld = rexp_ld;
  a.lb_k0 = k0; a.k_shared = k_shared;
  if (ctx->gemm_timer) { a.timer = ctx->gemm_timer; a.timer_role = 2; }
  const int S = ctx->S, Ad = ctx->A;
  a.shift = ctx->d_norm + 2 * S + 2 * Ad;  // mu_d
  a.scale = ctx->d_norm + 3 * S + 2 * Ad;  // sd_d
  const hipStream_t s = (hipStream_t)stream;
  // weight rows are padded to round_up(S, 128) (amx_layout n_out_pad): one 128 / 224 / 256-wide
  // column tile, or 128-wide column tiles
  const int n32 = amx::round_up(n_valid, 32), npad = amx::round_up(n_valid, 128);
  const int bn = n32 <= 128 ? 128 : n32 <= 224 ? 224 : n32 <= 256 ? 256 : 128;
  a.N = bn == 128 ? npad : bn;
  AMX_CHECK_ARG(strideW2 >= 2LL * K * a.N || groups == 1, "amx_gemm_out_unnorm_lb: strideW2=%lld", strideW2);
  lb_use_streamk(ctx, a, rows / 128 * (a.N / bn) * groups, 128, bn);
  if (ctx->lb_stage == 1) {
    switch (bn) {
      case 224: return launch_lb<EPI_UNNORM, LBOutDma<7>>(a, s);
      case 256: return launch_lb<EPI_UNNORM, LBOutDma<8>>(a, s);
      default: return launch_lb<EPI_UNNORM, LBOutDma<4>>(a, s);
    }
  }
  switch (bn) {
    case 224: return launch_lb<EPI_UNNORM, LBOut<224>>(a, s);
    case 256: return launch_lb<EPI_UNNORM, LBOut<256>>(a, s);
    default: return launch_lb<EPI_UNNORM, LBOut<128>>(a, s);
  }
}

// split-K scratch the lb launches may need (amx_split_workspace_floats takes the max with it)
long long amx::lb_split_floats(const amx_ctx* ctx, int groups, int rows, int* n_counters) {
  if (!ctx || groups < 1 || rows <= 0 || rows % 128 != 0) return 0;
  long long f = 0;
  int nc = 0, nwg = 0, ksplit = 0;
  const int K = ctx->ldk;
  const int n32 = amx::round_up(ctx->S, 32), npad = amx::round_up(ctx->S, 128);
  const int bn = n32 <= 128 ? 128 : n32 <= 224 ? 224 : n32 <= 256 ? 256 : 128;
  const int to = rows / 128 * ((bn == 128 ? npad : bn) / bn) * groups;
  if (lb_streamk(ctx, to, K / 32, &nwg, &ksplit)) {
    f = (long long)to * ksplit * 128 * bn;
    nc = to;
  }
  if (ctx->H % 256 == 0 && ctx->L > 1) {
    const int th = rows / 128 * (ctx->H / 256) * groups;
    if (2 * th < ctx->n_cus && lb_streamk(ctx, th, (ctx->k0_pad + (ctx->L - 1) * ctx->H) / 32, &nwg, &ksplit)) {
      const long long fh = (long long)th * ksplit * 128 * 256;
      f = f > fh ? f : fh;
      nc = nc > th ? nc : th;
    }
  }
  if (n_counters) *n_counters = nc;
  return f;
}

extern "C" int amx_set_lb_stage(amx_ctx* ctx, int stage) {
  AMX_CHECK_ARG(ctx, "amx_set_lb_stage: null ctx");
  AMX_CHECK_ARG(stage == 0 || stage == 1, "amx_set_lb_stage: stage=%d not in 0..1", stage);
  ctx->lb_stage = stage;
  return AMX_OK;
}
