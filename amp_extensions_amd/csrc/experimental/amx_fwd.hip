// The whole f16x3 ensemble forward in ONE launch (BasicMLP.forward over the dense-concat rows,
// milo/milo/dynamics.py:422-433, + DynamicsModel.forward's un-normalisation :231-232), for the
// lane counts whose row blocks fill the CUs exactly (the N = 1 rollout's 8192 lanes, the
// N = 8 share's 5120, ...).
//
// Why one launch.  The per-layer launches (amx_gemm_bias_act_h3 x L + amx_gemm_out_unnorm_h3)
// split every row of the dense-concat x0 | h0 | ... | h_{L-1} over two 256-column tiles, so
// each layer waits for the whole grid of the previous one.  Phase stamps of those launches
// (tools/h3_trace.py, profiles/r05h_h3_trace.txt) put 4.2-5.9 us of dispatch gap before every
// layer, 1.7-2.4 us of row-exponent prologue, and 1-9 us of grid-wide straggler tail after its
// K loop: ~60 us of a 315 us forward at the share, ~95 of 526 at 8192 lanes.
// Here a workgroup owns a block of BM rows of one member for ALL layers and all 512 hidden
// columns (8 waves x 64 columns), so no layer needs another workgroup's output: no grid-wide
// step between layers, no atomics, nothing for a workgroup to wait on but its own waves.
//
// Layout per workgroup (BM = 16 MB rows, MB = 4..6, one workgroup per CU):
//   * A (the dense rows, fp32 in HBM) is staged through LDS per 32-deep K-tile exactly as the
//     per-layer tiles stage it (row exponent scale, two fp16 limbs, 80-f16 rows), double-buffered,
//     one barrier per K-tile; every wave reads the same A fragments;
//   * W is NOT staged: each wave's 64 weight rows are read by that wave only, so the wave loads
//     its own MFMA fragments straight from L2 into registers (8 x 16 B per lane and K-tile, two
//     K-tiles in flight) from a fragment-ordered copy of the amx_split_f16x2 image
//     (amx_fwd_weight_image: each load one contiguous 1 KB) -- the LDS holds A only (40 KB at
//     BM = 128) and per K-tile the LDS traffic drops to the A fragments;
//   * the MFMA sequence of every 16 x 16 block is the per-layer tiles' (K-tiles in order, the
//     three limb products small terms first, v_mfma_f32_16x16x32_f16), and the row exponents
//     are the same (max over the slices read so far), so the result is bit-identical to the
//     per-layer launches (tests/test_gpu_fwd.py);
//   * the row exponents live in LDS: slot 0 (x0) is read once, each hidden layer's epilogue
//     max-es its slice's |h| bits into LDS (ds_max) and the running max is updated between
//     layers (slots 1..L are still written to row_exp, as the per-layer launches leave them);
//   * between layers: the next layer's first A / W tiles are loaded before this layer's
//     epilogue (their latency hides under it), the epilogue's stores are drained
//     (s_waitcnt vmcnt(0): the slice is in memory before any wave reads it back), two barriers.
// The output layer (N = n_out_pad = 256 or 128 weight rows, 8 waves x 32 or 16 columns) reads
// all L slices, un-normalises (two roundings, as torch's (y*scale)+mean) and writes preds.
// Workgroup -> (member, row block) through the XCD map (xcd_logical): an XCD's workgroups are
// consecutive row blocks of one member, so its L2 holds one member's weight panels.
#include "amx_common.h"
#include "amx_h3.h"

#include <type_traits>

// FW_CT (A/B builds): 1 = every 16 x 16 block computed transposed (the weight fragment in the
// MFMA's A slot): a lane then holds 4 consecutive COLUMNS of one row, so the hidden epilogue
// writes 16-B stores (4x fewer store instructions than the row-major block's 4-byte ones) and
// the row maxima need two lane exchanges instead of a reduce-scatter.  The k-sum inside the
// MFMA is the same for swapped operands, so the bits are the same (tests/test_gpu_fwd.py).
#ifndef FW_CT
#define FW_CT 1
#endif

// FW_DRAIN (A/B builds): 1 = every wave drains its epilogue stores (s_waitcnt vmcnt(0)) before
// the barrier that ends a layer; 0 = not: the slice is first read back 8 or more K-tiles into a
// later layer, and every wave has by then waited (vmcnt) for loads it issued after its stores --
// the VM counter retires in issue order on gfx9 -- and passed a barrier since
#ifndef FW_DRAIN
#define FW_DRAIN 0
#endif

// FW_TRACE (diagnostic builds, tools/fwd_trace.py): thread 0 of every workgroup stamps the
// device realtime clock (100 MHz) per layer: K loop entered, K loop done, layer done (after the
// epilogue and the exponent update) into fw_trace_buf[block][layer][3]
#ifndef FW_TRACE
#define FW_TRACE 0
#endif
#define FW_TRACE_L 9
#if FW_TRACE
__device__ unsigned long long fw_trace_buf[1024][FW_TRACE_L][3];
#define FW_STAMP(l, ph)                                                                        \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && (l) < FW_TRACE_L)                            \
      fw_trace_buf[blockIdx.x][(l)][(ph)] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
extern "C" int amx_fwd_trace_read(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(fw_trace_buf), sizeof(fw_trace_buf)) == hipSuccess ? 0 : -1;
}
#else
#define FW_STAMP(l, ph) \
  do {                  \
  } while (0)
#endif

// FW_NOUTER (A/B builds): 1 = the n-outer K-tile schedule (see ktile); 0 = m-outer
#ifndef FW_NOUTER
#define FW_NOUTER 1
#endif

namespace {

constexpr int FW_NT = 512;   // 8 waves, two per SIMD
constexpr int FW_BK = 32;    // K per K-tile (one v_mfma_f32_16x16x32_f16 deep)
constexpr int FW_LD = 80;    // f16 per LDS A row: [granule 0: limb0 16 | limb1 16 | granule 1 ...] + 16 pad
constexpr int FW_MAXL = 8;   // hidden layers supported
constexpr int FW_H = 512;    // hidden width (8 waves x 64 columns)

struct FwdArgs {
  const float* A; long long strideA; int lda;  // dense rows [g][rows][lda]: x0 | h0 | ... (slices written here)
  float* C;                                    // = A
  int k0, L, k_shared;                         // x0 columns (multiple of 32), hidden layers, shared x0 columns
  int rblocks;                                 // row blocks per member (rows / BM)
  const uint16_t* W2[FW_MAXL + 1];             // per layer: [g][N][K/16][2][16], group stride N*2K
  const int* wexp[FW_MAXL + 1];                // [g][N]
  const float* bias[FW_MAXL + 1];              // [g][N]
  int n_out, n_pad;                            // S, output weight rows (256 or 128)
  const float* scale; const float* shift;      // sd_d, mu_d
  float* preds; int ldp; long long strideP;
  int* row_exp; long long strideRexp; long long rexp_ld;  // [g][slot][rows]
  uint64_t* timer;                             // amx_set_gemm_timer buffer or null
};

typedef _Float16 hf8 __attribute__((ext_vector_type(8)));

}  // namespace

template <int MB, int NBO>
__global__ __launch_bounds__(FW_NT, 1) void k_forward_h3(FwdArgs a) {
  constexpr int BM = MB * 16;
  constexpr int NA = BM * 8;  // 16-B chunks of an A K-tile (8 per row)
  constexpr int VA = (NA + FW_NT - 1) / FW_NT;
  constexpr int NBH = 4;      // hidden: 4 column blocks of 16 per wave
  __shared__ __attribute__((aligned(16))) uint16_t sA[2 * BM * FW_LD];
  // running row exponents by layer parity (layer l stages and scales with sE[l & 1]), each hidden
  // layer's |h| row maxima (sMax[l], zeroed once), and the epilogue's bias / column exponents by
  // layer parity (staged one layer ahead): one barrier per layer boundary
  __shared__ __attribute__((aligned(16))) int sE[2][BM];
  __shared__ uint32_t sMax[FW_MAXL][BM];
  __shared__ __attribute__((aligned(16))) float sBias[2][FW_H];
  __shared__ __attribute__((aligned(16))) int sWexp[2][FW_H];

  if (a.timer && blockIdx.x == 0 && threadIdx.x == 0) a.timer[0] = __builtin_amdgcn_s_memrealtime();
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lc = lane & 15, lq = lane >> 4;
  const int logical = xcd_logical((int)gridDim.x, (int)blockIdx.x);
  const int g = logical / a.rblocks, rb = logical - g * a.rblocks;
  const long long rowbase = (long long)rb * BM;
  int* const rexp_g = a.row_exp + (long long)g * a.strideRexp;

  for (int r = t; r < BM; r += FW_NT) sE[0][r] = rexp_g[rowbase + r];  // slot 0: x0
  for (int e = t; e < FW_MAXL * BM; e += FW_NT) (&sMax[0][0])[e] = 0u;
  // bias / column exponents: layer 0's into LDS now, layer l + 1's loaded into registers while
  // layer l runs and stored into LDS at its epilogue
  auto layer_n = [&](int l) { return l < a.L ? FW_H : a.n_pad; };
  float pb = 0.f;
  int pe = 0;
  auto load_bias = [&](int l) {
    if (l <= a.L && t < layer_n(l)) {
      pb = a.bias[l][(long long)g * layer_n(l) + t];
      pe = a.wexp[l][(long long)g * layer_n(l) + t];
    }
  };
  auto store_bias = [&](int l) {
    if (l <= a.L && t < layer_n(l)) {
      sBias[l & 1][t] = pb;
      sWexp[l & 1][t] = pe;
    }
  };
  load_bias(0);
  store_bias(0);

  // A staging map (as h3_tile's M16 tiles): chunk q = t + 512 j -> row q / 8, k 4 (q % 8)
  int a_src[VA], a_dst[VA], a_row[VA], a_sh[VA];
  bool a_ok[VA];
#pragma unroll
  for (int j = 0; j < VA; ++j) {
    const int q = t + FW_NT * j;
    a_ok[j] = (NA % FW_NT == 0 || j + 1 < VA) ? true : q < NA;
    const int r = a_ok[j] ? q / 8 : 0, c = q % 8;
    a_src[j] = r * a.lda + 4 * c;
    a_dst[j] = r * FW_LD + (c >> 2) * 32 + (c & 3) * 4;
    a_row[j] = r;
  }
  const float* Ag = a.A + (long long)g * a.strideA + rowbase * a.lda;
  const float* Ag0 = a.A + rowbase * a.lda;  // group 0's rows: the shared x0 columns
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Ag), 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsA0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Ag0), 0, 0x7ffffff0, 0x00020000);
  const int nks = a.k_shared / FW_BK;

  f32x4 ra[VA], rn[VA];  // A stage registers: the next tile to publish, the one after
  auto loadA = [&](f32x4 (&dst)[VA], int kt) {
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok[j])
        dst[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(kt < nks ? rsA0 : rsA, a_src[j] * 4,
                                                                                 kt * FW_BK * 4, 0));
  };
  auto publish = [&](const f32x4 (&src)[VA], int buf) {
    uint16_t* base = sA + buf * (BM * FW_LD);
#pragma unroll
    for (int j = 0; j < VA; ++j)
      if (a_ok[j]) {
        f32x4 x = src[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_ldexpf(x[i], a_sh[j]);
        u32x2 l0, l1;
        split2(x, l0, l1);
        *reinterpret_cast<u32x2*>(base + a_dst[j]) = l0;
        *reinterpret_cast<u32x2*>(base + a_dst[j] + 16) = l1;
      }
  };
  // layer l's staging scale: layer l-1's exponents (sE[(l-1) & 1], stable) max-ed with its
  // slice's maxima -- sE[l & 1] itself is being written in the same phase
  auto set_shifts = [&](int l) {
#pragma unroll
    for (int j = 0; j < VA; ++j) {
      int e = sE[l > 0 ? (l - 1) & 1 : 0][a_row[j]];
      if (l > 0) {
        const int e1 = exp_of_bits(sMax[l - 1][a_row[j]]);
        e = e1 > e ? e1 : e;
      }
      a_sh[j] = HSC - e;
    }
  };

  // W fragments from the fragment-ordered image (amx_fwd_weight_image): the 16 B lane l needs for
  // column block b (16 weight rows), K-tile kt and limb L sit at ((b * nk + kt) * 2 + L) * 1 KB +
  // 16 l, so every fragment load is one contiguous 1 KB (the row-major image's 16 rows 4.6-9 KB
  // apart stalled the L1 on tag conflicts: TCP_READ_TAGCONFLICT_STALL_CYCLES, profiles/r05j_*)
  hf8 gb[2][NBH][2];
  __amdgpu_buffer_rsrc_t rsW;
  int K = 0, nk = 0, cb16 = 0;
  auto setW = [&](int l, int ncols_wave) {
    K = l < a.L ? a.k0 + l * FW_H : a.k0 + a.L * FW_H;
    nk = K / FW_BK;
    const int N = l < a.L ? FW_H : a.n_pad;
    const uint16_t* Wg = a.W2[l] + (long long)g * N * 2 * K;
    rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Wg), 0, 0x7ffffff0, 0x00020000);
    cb16 = wave * ncols_wave / 16;
  };
  const int w_lane = lane * 16;
  auto loadW = [&](auto par, auto nb, int kt) {
    constexpr int P = decltype(par)::value, NB = decltype(nb)::value;
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int l = 0; l < 2; ++l)
        gb[P][n][l] = __builtin_bit_cast(
            hf8, __builtin_amdgcn_raw_buffer_load_b128(rsW, w_lane, (((cb16 + n) * nk + kt) * 2 + l) * 1024, 0));
  };

  f32x4 acc[MB][NBH];
  const int koff = (lane >> 5) * 32 + ((lane >> 4) & 1) * 8;  // the lane's k within an LDS A row
  const uint16_t* const a_frag = sA + lc * FW_LD + koff;
  // one K-tile (parity P: LDS buffer P, W registers gb[P])
  auto ktile = [&](auto par, auto nb, int kt) {
    constexpr int P = decltype(par)::value, NB = decltype(nb)::value;
    __syncthreads();  // A tile kt visible in buffer P; buffer P^1 (tile kt-1) fully read
    const uint16_t* As = a_frag + P * (BM * FW_LD);
    const int kn = kt + 2 < nk ? kt + 2 : nk - 1;
#if FW_NOUTER
    {
      // n-outer over halves of the m-blocks (the whole tile at MB <= 5): the half's A fragments
      // read up front, then per column block n its MFMAs; in the last half block n's W registers
      // are dead after its MFMAs, so its loads for tile kt + 2 go right behind them, and the A
      // publish / loads sit between the first blocks (the MFMA pipe never waits on a staging
      // phase).  Every accumulator still sees p = 0, 1, 2 per K-tile in K-tile order.
      constexpr int MH = MB <= 5 ? MB : (MB + 1) / 2, NH = (MB + MH - 1) / MH;
      constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        hf8 gaa[MH][2];
#pragma unroll
        for (int mm = 0; mm < MH; ++mm)
#pragma unroll
          for (int l = 0; l < 2; ++l)
            if (h * MH + mm < MB)
              gaa[mm][l] = *reinterpret_cast<const hf8*>(As + (h * MH + mm) * 16 * FW_LD + l * 16);
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int mm = 0; mm < MH; ++mm) {
            const int m = h * MH + mm;
            if (m < MB) {
#pragma unroll
              for (int p = 0; p < 3; ++p)
#if FW_CT
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gb[P][n][PB[p]], gaa[mm][PA[p]], acc[m][n], 0, 0, 0);
#else
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gaa[mm][PA[p]], gb[P][n][PB[p]], acc[m][n], 0, 0, 0);
#endif
            }
          }
          __builtin_amdgcn_sched_barrier(0);
          if (h == 0 && n == 0) publish(ra, P ^ 1);
          if (h == 0 && n == (NB > 1 ? 1 : 0)) loadA(ra, kn);
          if (h == NH - 1) {
#pragma unroll
            for (int l = 0; l < 2; ++l)
              gb[P][n][l] = __builtin_bit_cast(
                  hf8, __builtin_amdgcn_raw_buffer_load_b128(rsW, w_lane, (((cb16 + n) * nk + kn) * 2 + l) * 1024, 0));
          }
        }
      }
      return;
    }
#endif
    hf8 ga[2][2];
    ga[0][0] = *reinterpret_cast<const hf8*>(As);
    ga[0][1] = *reinterpret_cast<const hf8*>(As + 16);
    // branch-free (a conditional load makes hipcc wait vmcnt(0) at the next publish): past the
    // end, tile nk - 1 is re-published into the free buffer and re-loaded
    publish(ra, P ^ 1);
    loadA(ra, kn);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      if (m + 1 < MB) {
#pragma unroll
        for (int l = 0; l < 2; ++l)
          ga[(m + 1) & 1][l] = *reinterpret_cast<const hf8*>(As + (m + 1) * 16 * FW_LD + l * 16);
      }
      __builtin_amdgcn_sched_barrier(0);
      constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};  // small terms first (as h3_tile)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int n = 0; n < NB; ++n)
#if FW_CT
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gb[P][n][PB[p]], ga[m & 1][PA[p]], acc[m][n], 0, 0, 0);
#else
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ga[m & 1][PA[p]], gb[P][n][PB[p]], acc[m][n], 0, 0, 0);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
    loadW(par, nb, kn);
  };
  auto klayer = [&](auto nb) {
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int n = 0; n < NBH; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; kt += 2) {  // nk is even (K % 64 == 0)
      ktile(std::integral_constant<int, 0>{}, nb, kt);
      ktile(std::integral_constant<int, 1>{}, nb, kt + 1);
    }
  };
  // the next layer's first tiles (A 0 -> rn... published after the exponents are updated)
  auto prefetch = [&](int l, auto nb) {
    setW(l, decltype(nb)::value * 16);
    loadA(rn, 0);
    loadA(ra, 1);
    loadW(std::integral_constant<int, 0>{}, nb, 0);
  };
  auto start = [&](int l, auto nb) {  // after the exponents: tile 0 into LDS buffer 0, W tile 1
    set_shifts(l);
    publish(rn, 0);
    loadW(std::integral_constant<int, 1>{}, nb, 1);
    load_bias(l + 1);
  };

  __syncthreads();  // sE, sMax, layer 0's bias
  prefetch(0, std::integral_constant<int, NBH>{});
  start(0, std::integral_constant<int, NBH>{});
  for (int l = 0; l < a.L; ++l) {
    FW_STAMP(l, 0);
    klayer(std::integral_constant<int, NBH>{});
    FW_STAMP(l, 1);
    const int col_off = K;  // this layer's slice starts at its own K
    const int par = l & 1;
    const int* const sEl = sE[par];
#if FW_CT
    f32x4 bv[NBH];  // columns n*16 + 4 lq .. + 3
    int4 ec[NBH];
#pragma unroll
    for (int n = 0; n < NBH; ++n) {
      const int col = wave * 64 + n * 16 + 4 * lq;
      bv[n] = *reinterpret_cast<const f32x4*>(&sBias[par][col]);
      ec[n] = *reinterpret_cast<const int4*>(&sWexp[par][col]);
    }
#else
    float bv[NBH];
    int ec[NBH];
#pragma unroll
    for (int n = 0; n < NBH; ++n) {
      const int col = wave * 64 + n * 16 + lc;
      bv[n] = sBias[par][col];
      ec[n] = sWexp[par][col] - 2 * HSC;
    }
#endif
    if (l + 1 < a.L) prefetch(l + 1, std::integral_constant<int, NBH>{});
    else prefetch(a.L, std::integral_constant<int, NBO>{});
    // epilogue: bias + ReLU into the slice, |h| row maxima into sMax
    {
      // buffer stores: the lane's offset in one VGPR, the row / column / block terms in SGPRs (64-bit
      // per-row addresses hoisted out of the layer loop spilled at BM = 128)
      const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc(
          a.C + (long long)g * a.strideA + rowbase * a.lda, 0, 0x7ffffff0, 0x00020000);
#if FW_CT
      const int c_lane = (lc * a.lda + wave * 64 + 4 * lq) * 4;
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const int er = sEl[m * 16 + lc] - 2 * HSC;
        uint32_t q = 0u;
#pragma unroll
        for (int n = 0; n < NBH; ++n) {
          f32x4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float x = __builtin_amdgcn_ldexpf(acc[m][n][i], er + ec[n][i]) + bv[n][i];
            x = (x < 0.f) ? 0.f : x;  // keeps NaN, as torch.relu
            v[i] = x;
            const uint32_t b = __float_as_uint(x) & 0x7fffffffu;
            q = q > b ? q : b;
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsC, c_lane,
                                                 (m * 16 * a.lda + col_off + n * 16) * 4, 0);
        }
        // max over the 4 lanes lq holding the row's other columns, then over the waves (ds_max)
        uint32_t o = (uint32_t)__shfl_xor((int)q, 16);
        q = q > o ? q : o;
        o = (uint32_t)__shfl_xor((int)q, 32);
        q = q > o ? q : o;
        if (lq == 0) atomicMax(&sMax[l][m * 16 + lc], q);
      }
#else
      const int c_lane = (4 * lq * a.lda + wave * 64 + lc) * 4;
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const int4 ev = *reinterpret_cast<const int4*>(sEl + m * 16 + 4 * lq);
        const int er[4] = {ev.x, ev.y, ev.z, ev.w};
        uint32_t q4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int n = 0; n < NBH; ++n) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = __builtin_amdgcn_ldexpf(acc[m][n][j], er[j] + ec[n]) + bv[n];
            v = (v < 0.f) ? 0.f : v;  // keeps NaN, as torch.relu
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsC, c_lane,
                                                  ((m * 16 + j) * a.lda + col_off + n * 16) * 4, 0);
            const uint32_t b = __float_as_uint(v) & 0x7fffffffu;
            q4[j] = q4[j] > b ? q4[j] : b;
          }
        }
        // max over the 16 column lanes of each of the lane's 4 rows (reduce-scatter over lc bits
        // 3, 2, then a full max over bits 1, 0), into sMax (ds_max)
        rs_step<8, 2>(q4, lc);
        rs_step<4, 1>(q4, lc);
        uint32_t o = (uint32_t)__builtin_amdgcn_ds_swizzle((int)q4[0], 0x1f | (2 << 10));
        q4[0] = q4[0] > o ? q4[0] : o;
        o = (uint32_t)__builtin_amdgcn_ds_swizzle((int)q4[0], 0x1f | (1 << 10));
        q4[0] = q4[0] > o ? q4[0] : o;
        if ((lc & 3) == 0) atomicMax(&sMax[l][m * 16 + 4 * lq + ((lc >> 3) & 1) * 2 + ((lc >> 2) & 1)], q4[0]);
      }
#endif
    }
    store_bias(l + 1);  // the next layer's bias / exponents (sBias[par ^ 1]: last read a layer ago)
#if FW_DRAIN
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slice is in memory before any wave reads it
#endif
    __syncthreads();  // sMax[l] complete; every wave is past its reads of sE[par ^ 1]
    for (int r = t; r < BM; r += FW_NT) {
      const int e = exp_of_bits(sMax[l][r]);
      rexp_g[(long long)(l + 1) * a.rexp_ld + rowbase + r] = e;
      const int o = sEl[r];
      sE[par ^ 1][r] = e > o ? e : o;  // read by layer l + 1's epilogue, K-tile barriers later
    }
    FW_STAMP(l, 2);
    if (l + 1 < a.L) start(l + 1, std::integral_constant<int, NBH>{});
    else start(l + 1, std::integral_constant<int, NBO>{});
  }
  // output layer: all L slices, NBO blocks of 16 columns per wave
  FW_STAMP(a.L, 0);
  klayer(std::integral_constant<int, NBO>{});
  FW_STAMP(a.L, 1);
  {
    const int par = a.L & 1;
    const int* const sEl = sE[par];
    const float* const bias = sBias[par];
    const int* const wexp = sWexp[par];
    const __amdgpu_buffer_rsrc_t rsP = __builtin_amdgcn_make_buffer_rsrc(
        a.preds + (long long)g * a.strideP + rowbase * a.ldp, 0, 0x7ffffff0, 0x00020000);
#if FW_CT
#pragma unroll
    for (int n = 0; n < NBO; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = wave * NBO * 16 + n * 16 + 4 * lq + i;
        if (col < a.n_out) {
          const float bv = bias[col];
          const float sc = a.scale[col], sh = a.shift[col];
          const int ec = wexp[col] - 2 * HSC;
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            const float y = __builtin_amdgcn_ldexpf(acc[m][n][i], sEl[m * 16 + lc] + ec) + bv;
            const float prod = y * sc;  // two roundings, as torch's (y*scale)+mean
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prod + sh), rsP, (lc * a.ldp + col) * 4,
                                                  m * 16 * a.ldp * 4, 0);
          }
        }
      }
    }
#else
#pragma unroll
    for (int n = 0; n < NBO; ++n) {
      const int col = wave * NBO * 16 + n * 16 + lc;
      if (col < a.n_out) {
        const float bv = bias[col];
        const float sc = a.scale[col], sh = a.shift[col];
        const int ec = wexp[col] - 2 * HSC;
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          const int4 ev = *reinterpret_cast<const int4*>(sEl + m * 16 + 4 * lq);
          const int er[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float y = __builtin_amdgcn_ldexpf(acc[m][n][j], er[j] + ec) + bv;
            const float prod = y * sc;  // two roundings, as torch's (y*scale)+mean
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prod + sh), rsP, (4 * lq * a.ldp + col) * 4,
                                                  (m * 16 + j) * a.ldp * 4, 0);
          }
        }
      }
    }
#endif
  }
#if FW_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  FW_STAMP(a.L, 2);
#endif
  if (a.timer) {  // as gemm_timer_end: the last workgroup adds (now - start)
    __syncthreads();
    if (threadIdx.x == 0) {
      if (atomicAdd(reinterpret_cast<unsigned long long*>(a.timer + 1), 1ull) == gridDim.x - 1) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        atomicAdd(reinterpret_cast<unsigned long long*>(a.timer + 2), (unsigned long long)(now - a.timer[0]));
        atomicAdd(reinterpret_cast<unsigned long long*>(a.timer + 3), 1ull);
        atomicExch(reinterpret_cast<unsigned long long*>(a.timer + 1), 0ull);
      }
    }
  }
}

// amx_fwd_weight_image: row-major amx_split_f16x2 image [g][N][K/16][2][16] -> fragment order
// [g][N/16][K/32][limb 2][lane 64][8]: lane l = 32 granule + 16 half + row (l & 15) of the block
__global__ __launch_bounds__(256) void k_fwd_weight_image(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          int N, int K, long long units) {
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u >= units) return;
  const int lane = (int)(u & 63);
  long long q = u >> 6;
  const int limb = (int)(q & 1);
  q >>= 1;
  const int nkt = K / 32, nb16 = N / 16;
  const int kt = (int)(q % nkt);
  q /= nkt;
  const int b = (int)(q % nb16);
  const long long g = q / nb16;
  const int row = b * 16 + (lane & 15), gi = lane >> 5, h = (lane >> 4) & 1;
  // source 16-B unit: f16 offset row * 2K + kt * 64 + gi * 32 + limb * 16 + h * 8
  const long long so = (g * N + row) * 2LL * K + kt * 64 + gi * 32 + limb * 16 + h * 8;
  dst[u] = src[so / 8];
}

extern "C" int amx_fwd_weight_image(amx_ctx* ctx, int groups, int N, int K, const uint16_t* W2, uint16_t* W2f,
                                    void* stream) {
  AMX_CHECK_ARG(ctx && W2 && W2f && W2 != W2f, "amx_fwd_weight_image: null or aliased argument");
  AMX_CHECK_ARG(groups >= 1 && N > 0 && N % 16 == 0 && K > 0 && K % 32 == 0,
                "amx_fwd_weight_image: groups=%d N=%d (multiple of 16) K=%d (multiple of 32)", groups, N, K);
  AMX_CHECK_ARG(amx::aligned16(W2) && amx::aligned16(W2f), "amx_fwd_weight_image: operands must be 16-byte aligned");
  const long long units = (long long)groups * N * K / 4;  // 16-B units (2 limbs x K f16 per row)
  if (units == 0) return AMX_OK;
  hipLaunchKernelGGL(k_fwd_weight_image, dim3((unsigned)((units + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint4*>(W2), reinterpret_cast<uint4*>(W2f), N, K, units);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

// rows per workgroup (16 MB) of the one-launch forward for this shape, 0 when it does not apply:
// one workgroup per CU of MB = 4..6 row blocks of 16 (64-96 rows).  At 128 rows (8192 lanes) the
// n-outer K-tile schedule does not fit the registers and the m-outer one ran 2.99 us per K-tile
// against the per-layer 256 x 256 tile's 2.6 (profiles/r05k_fwd_trace.txt); two rounds of
// 64-row workgroups read every weight twice -- those shapes keep the per-layer launches.
static int fwd_mb(const amx_ctx* ctx, int groups, int rows) {
  if (ctx->n_cus <= 0 || rows % 16 != 0) return 0;
  const long long blocks = (long long)groups * (rows / 16);
  if (blocks % ctx->n_cus != 0) return 0;
  const long long q = blocks / ctx->n_cus;  // 16-row blocks per CU: one workgroup of q blocks per CU
  return (q >= 4 && q <= 6 && rows % (16 * q) == 0) ? (int)q : 0;
}

extern "C" int amx_forward_h3_rows(amx_ctx* ctx, int groups, int rows) {
  if (!ctx || groups < 1 || rows < 1) return 0;
  return 16 * fwd_mb(ctx, groups, rows);
}

extern "C" int amx_forward_h3(amx_ctx* ctx, int groups, int rows, int k0, int hidden, int n_hidden, float* A,
                              int lda, long long strideA, const uint16_t* const* W2, const int* const* w_exp,
                              const float* const* bias, int n_out_pad, float* preds, int ldp, long long strideP,
                              int* row_exp, long long strideRexp, int k_shared, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "amx_forward_h3: null ctx or no normalizers");
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS, "amx_forward_h3: groups=%d", groups);
  AMX_CHECK_ARG(hidden == FW_H, "amx_forward_h3: hidden=%d (the one-launch forward is built for %d)", hidden, FW_H);
  AMX_CHECK_ARG(n_hidden >= 1 && n_hidden <= FW_MAXL, "amx_forward_h3: n_hidden=%d (1..%d)", n_hidden, FW_MAXL);
  AMX_CHECK_ARG(k0 > 0 && k0 % 64 == 0, "amx_forward_h3: k0=%d must be a positive multiple of 64", k0);
  AMX_CHECK_ARG(k_shared == 0 || k_shared == k0, "amx_forward_h3: k_shared=%d must be 0 or k0", k_shared);
  const int kout = k0 + n_hidden * hidden;
  AMX_CHECK_ARG(lda >= kout && lda % 4 == 0, "amx_forward_h3: lda=%d < %d or not a multiple of 4", lda, kout);
  AMX_CHECK_ARG(strideA >= (long long)rows * lda || groups == 1, "amx_forward_h3: strideA=%lld", strideA);
  AMX_CHECK_ARG(n_out_pad == 256 || n_out_pad == 128, "amx_forward_h3: n_out_pad=%d (256 or 128)", n_out_pad);
  AMX_CHECK_ARG(ctx->S <= n_out_pad && ctx->S > n_out_pad - 128, "amx_forward_h3: S=%d vs n_out_pad=%d", ctx->S,
                n_out_pad);
  AMX_CHECK_ARG(A && preds && row_exp && W2 && w_exp && bias, "amx_forward_h3: null argument");
  AMX_CHECK_ARG(amx::aligned16(A), "amx_forward_h3: A must be 16-byte aligned");
  AMX_CHECK_ARG(ldp >= ctx->S, "amx_forward_h3: ldp=%d < S=%d", ldp, ctx->S);
  AMX_CHECK_ARG(strideRexp >= (long long)(n_hidden + 1) * rows || groups == 1, "amx_forward_h3: strideRexp=%lld",
                strideRexp);
  const int mb = fwd_mb(ctx, groups, rows);
  AMX_CHECK_ARG(mb > 0, "amx_forward_h3: groups=%d x rows=%d do not make one whole CU round of 64..96-row blocks "
                "(amx_forward_h3_rows returns 0; use the per-layer launches)", groups, rows);
  FwdArgs a = {};
  a.A = A; a.C = A; a.strideA = strideA; a.lda = lda;
  a.k0 = k0; a.L = n_hidden; a.k_shared = k_shared;
  a.rblocks = rows / (16 * mb);
  for (int l = 0; l <= n_hidden; ++l) {
    AMX_CHECK_ARG(W2[l] && w_exp[l] && bias[l], "amx_forward_h3: null layer %d operand", l);
    AMX_CHECK_ARG(amx::aligned16(W2[l]), "amx_forward_h3: W2[%d] must be 16-byte aligned", l);
    a.W2[l] = W2[l]; a.wexp[l] = w_exp[l]; a.bias[l] = bias[l];
  }
  a.n_out = ctx->S; a.n_pad = n_out_pad;
  const int S = ctx->S, Ad = ctx->A;
  a.shift = ctx->d_norm + 2 * S + 2 * Ad;  // mu_d
  a.scale = ctx->d_norm + 3 * S + 2 * Ad;  // sd_d
  a.preds = preds; a.ldp = ldp; a.strideP = strideP;
  a.row_exp = row_exp; a.strideRexp = strideRexp; a.rexp_ld = rows;
  a.timer = ctx->gemm_timer;
  const int nwg = groups * a.rblocks;
  const hipStream_t s = (hipStream_t)stream;
#define AMX_FWD_LAUNCH(MB_, NBO_) hipLaunchKernelGGL((k_forward_h3<MB_, NBO_>), dim3(nwg), dim3(FW_NT), 0, s, a)
#define AMX_FWD_CASE(MB_)                                \
  case MB_:                                              \
    if (n_out_pad == 256) AMX_FWD_LAUNCH(MB_, 2);        \
    else AMX_FWD_LAUNCH(MB_, 1);                         \
    break;
  switch (mb) {
    AMX_FWD_CASE(4)
    AMX_FWD_CASE(5)
    AMX_FWD_CASE(6)
    default: break;
  }
#undef AMX_FWD_CASE
#undef AMX_FWD_LAUNCH
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
