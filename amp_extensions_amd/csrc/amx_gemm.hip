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
// Tile: 128x128 per workgroup, BK = 32, 4 waves in 2x2, each wave 64x64 = 2x2 MFMA
// 32x32 tiles.  Operands are register-staged through LDS (double buffer, one barrier per
// K-tile).  Lane l of an MFMA supplies k-slot h = l>>5; we map slot h of MFMA step s to
// k = 16h + s so that each lane reads 16 consecutive floats of its row with 4
// ds_read_b128 (the same permutation on A and W keeps the contraction exact).  LDS rows
// are padded to 36 floats: rows 16 apart land on distinct 16-byte bank slots, so the
// 16-lane groups of ds_read_b128 are conflict-free.
#include "amx_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 32;
constexpr int LDS_LD = BK + 4;                          // floats per LDS row
constexpr int TILE_FLOATS = (BM + BN) * LDS_LD;         // one stage (A + W)
constexpr size_t LDS_BYTES = 2 * TILE_FLOATS * sizeof(float);  // 73,728 B: 2 WGs per CU

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
};

// Linear block id -> (group, tile_m, tile_n).  Workgroups are dispatched round-robin over
// the 8 XCDs, so block ids congruent mod 8 share an L2.  We hand each XCD a contiguous
// run of logical tiles (tile_n fastest: consecutive tiles reuse the same A row panel;
// then tile_m: they reuse the same weight panels of one ensemble member).  Bijective for
// any tile count (cdna_hip_programming.md T1).
__device__ inline void map_tile(const GemmArgs& a, int& g, int& tm, int& tn) {
  const int nwg = a.tiles_m * a.tiles_n * a.groups;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int logical = base + (orig >> 3);
  tn = logical % a.tiles_n;
  const int rest = logical / a.tiles_n;
  tm = rest % a.tiles_m;
  g = rest / a.tiles_m;
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm_nt(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int g, tm, tn;
  map_tile(a, g, tm, tn);

  const float* __restrict__ Ag = a.A + (long long)g * a.strideA + (long long)tm * BM * a.lda;
  const float* __restrict__ Wg = a.W + (long long)g * a.strideW + (long long)tn * BN * a.ldw;

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;

  // staging map: float4 index q = t + 256*j (j < 4) -> row q>>3, column 4*(q&7).
  // The stage registers are named scalars (not an array captured by a lambda: that put
  // them in scratch and made every iteration wait for its own prefetch).
  const int st_r = t >> 3, st_c = (t & 7) * 4;
  const float* a_src = Ag + (long long)st_r * a.lda + st_c;
  const float* w_src = Wg + (long long)st_r * a.ldw + st_c;
  const long long a_step = 32LL * a.lda, w_step = 32LL * a.ldw;
  float* const a_dst0 = smem + st_r * LDS_LD + st_c;
  float* const w_dst0 = smem + BM * LDS_LD + st_r * LDS_LD + st_c;

  float4 ra0, ra1, ra2, ra3, rw0, rw1, rw2, rw3;
#define AMX_GLOAD(k0)                                                             \
  do {                                                                            \
    ra0 = *reinterpret_cast<const float4*>(a_src + (k0));                         \
    ra1 = *reinterpret_cast<const float4*>(a_src + a_step + (k0));                \
    ra2 = *reinterpret_cast<const float4*>(a_src + 2 * a_step + (k0));            \
    ra3 = *reinterpret_cast<const float4*>(a_src + 3 * a_step + (k0));            \
    rw0 = *reinterpret_cast<const float4*>(w_src + (k0));                         \
    rw1 = *reinterpret_cast<const float4*>(w_src + w_step + (k0));                \
    rw2 = *reinterpret_cast<const float4*>(w_src + 2 * w_step + (k0));            \
    rw3 = *reinterpret_cast<const float4*>(w_src + 3 * w_step + (k0));            \
  } while (0)
#define AMX_LSTORE(buf)                                                           \
  do {                                                                            \
    float* ad = a_dst0 + (buf) * TILE_FLOATS;                                     \
    float* wd = w_dst0 + (buf) * TILE_FLOATS;                                     \
    *reinterpret_cast<float4*>(ad) = ra0;                                         \
    *reinterpret_cast<float4*>(ad + 32 * LDS_LD) = ra1;                           \
    *reinterpret_cast<float4*>(ad + 64 * LDS_LD) = ra2;                           \
    *reinterpret_cast<float4*>(ad + 96 * LDS_LD) = ra3;                           \
    *reinterpret_cast<float4*>(wd) = rw0;                                         \
    *reinterpret_cast<float4*>(wd + 32 * LDS_LD) = rw1;                           \
    *reinterpret_cast<float4*>(wd + 64 * LDS_LD) = rw2;                           \
    *reinterpret_cast<float4*>(wd + 96 * LDS_LD) = rw3;                           \
  } while (0)

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = a.K / BK;
  AMX_GLOAD(0);
  AMX_LSTORE(0);
  __syncthreads();

  const int a_off = (wm * 64 + li) * LDS_LD + lh * 16;
  const int w_off = BM * LDS_LD + (wn * 64 + li) * LDS_LD + lh * 16;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // prefetch the next K-tile (the last iteration re-reads its own tile: branch-free loop)
    const int kn = (kt + 1 < nk ? kt + 1 : kt) * BK;
    AMX_GLOAD(kn);
    // keep the prefetch ahead of the MFMA block (hipcc otherwise sinks the loads to their
    // consumer, the LDS store after the MFMAs, and the latency is exposed every K-tile)
    __builtin_amdgcn_sched_barrier(0);

    const float* As = smem + cur * TILE_FLOATS + a_off;
    const float* Ws = smem + cur * TILE_FLOATS + w_off;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float4 fa0 = *reinterpret_cast<const float4*>(As + v * 4);
      const float4 fa1 = *reinterpret_cast<const float4*>(As + 32 * LDS_LD + v * 4);
      const float4 fb0 = *reinterpret_cast<const float4*>(Ws + v * 4);
      const float4 fb1 = *reinterpret_cast<const float4*>(Ws + 32 * LDS_LD + v * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a0 = fa0[e], a1 = fa1[e];
        const float b0 = fb0[e], b1 = fb1[e];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    AMX_LSTORE(cur ^ 1);
    __syncthreads();
  }
#undef AMX_GLOAD
#undef AMX_LSTORE

  // ---- epilogue ---------------------------------------------------------------------
  // C/D map of 32x32 f32 MFMA: column = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
  const int row0 = tm * BM + wm * 64;
  const int col0 = tn * BN + wn * 64;

  if constexpr (EPI == EPI_BIAS_ACT) {
    const float* bias = a.bias + (long long)g * a.strideBias;
    float* Cg = a.C + (long long)g * a.strideC;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int col = col0 + n * 32 + li;
      const float bv = bias[col];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
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
    for (int n = 0; n < 2; ++n) {
      const int col = col0 + n * 32 + li;
      if (col < a.n_valid) {
        const float bv = bias[col];
        const float sc = a.scale[col], sh = a.shift[col];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
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
  } else {  // EPI_RFF
    // Stage the raw 128x128 tile through LDS, then one column per thread: coalesced phi
    // rows, one (non-unrolled) cos call site instead of 64 inlined copies, and the fp64
    // column sum of the valid rows in fixed row order (deterministic).
    constexpr int CLD = BN + 4;
    float* Cs = smem;  // [BM][CLD] = 67,584 B, reuses the stage buffers (last barrier passed)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = wm * 64 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          Cs[r * CLD + wn * 64 + n * 32 + li] = acc[m][n][e];
        }
    __syncthreads();
    const int c = t & (BN - 1), half = t >> 7;
    const int col = tn * BN + c;
    const float bv = a.bias[col];
    double csum = 0.0;
    float* Cg = a.C;
#pragma unroll 2
    for (int i = 0; i < BM / 2; ++i) {
      const int r = half * (BM / 2) + i;
      const int row = tm * BM + r;
      const float z = Cs[r * CLD + c] + bv;       // nn.Linear: x W^T + b
      const float phi = cosf(z) * a.rff_scale;   // torch.cos(.) * np.sqrt(2/F)
      Cg[(long long)row * a.ldc + col] = phi;
      const bool valid = row < a.n_valid && (a.row_mask == nullptr || a.row_mask[row] != 0);
      csum += valid ? (double)phi : 0.0;
    }
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);
    if (half == 1) red[c] = csum;
    __syncthreads();
    if (half == 0) a.col_partials[(long long)tm * a.N + col] = csum + red[c];
  }
}

int launch_gemm(int epi, GemmArgs& a, hipStream_t stream) {
  a.tiles_m = a.rows / BM;
  a.tiles_n = (epi == EPI_UNNORM) ? amx::round_up(a.n_valid, BN) / BN : a.N / BN;
  const int nwg = a.tiles_m * a.tiles_n * a.groups;
  if (nwg == 0) return AMX_OK;
  dim3 grid(nwg), block(256);
  switch (epi) {
    case EPI_BIAS_ACT:
      hipLaunchKernelGGL(k_gemm_nt<EPI_BIAS_ACT>, grid, block, LDS_BYTES, stream, a);
      break;
    case EPI_UNNORM:
      hipLaunchKernelGGL(k_gemm_nt<EPI_UNNORM>, grid, block, LDS_BYTES, stream, a);
      break;
    default:
      hipLaunchKernelGGL(k_gemm_nt<EPI_RFF>, grid, block, LDS_BYTES, stream, a);
      break;
  }
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

int check_common(const char* fn, int groups, int rows, int K, const float* A, int lda, const float* W,
                 int ldw) {
  AMX_CHECK_ARG(groups >= 1 && groups <= AMX_MAX_MODELS, "%s: groups=%d", fn, groups);
  AMX_CHECK_ARG(rows >= 0 && rows % BM == 0, "%s: rows=%d must be a multiple of %d", fn, rows, BM);
  AMX_CHECK_ARG(K > 0 && K % BK == 0, "%s: K=%d must be a positive multiple of %d", fn, K, BK);
  AMX_CHECK_ARG(A && W, "%s: null operand", fn);
  AMX_CHECK_ARG(amx::aligned16(A) && amx::aligned16(W), "%s: operands must be 16-byte aligned", fn);
  AMX_CHECK_ARG(lda >= K && lda % 4 == 0, "%s: lda=%d (K=%d) must be >= K and a multiple of 4", fn, lda, K);
  AMX_CHECK_ARG(ldw >= K && ldw % 4 == 0, "%s: ldw=%d (K=%d) must be >= K and a multiple of 4", fn, ldw, K);
  return AMX_OK;
}

}  // namespace

extern "C" int amx_gemm_bias_act(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                                 long long strideA, const float* W, int ldw, long long strideW,
                                 const float* bias, long long strideBias, float* C, int ldc, long long strideC,
                                 int col_off, int act, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_gemm_bias_act: null ctx");
  int rc = check_common("amx_gemm_bias_act", groups, rows, K, A, lda, W, ldw);
  if (rc) return rc;
  AMX_CHECK_ARG(N > 0 && N % BN == 0, "amx_gemm_bias_act: N=%d must be a multiple of %d", N, BN);
  AMX_CHECK_ARG(bias && C, "amx_gemm_bias_act: null bias/C");
  AMX_CHECK_ARG(col_off >= 0 && col_off + N <= ldc, "amx_gemm_bias_act: col_off=%d N=%d ldc=%d", col_off, N, ldc);
  AMX_CHECK_ARG(act == AMX_ACT_NONE || act == AMX_ACT_RELU, "amx_gemm_bias_act: act=%d", act);
  GemmArgs a = {};
  a.A = A; a.strideA = strideA; a.lda = lda;
  a.W = W; a.strideW = strideW; a.ldw = ldw;
  a.bias = bias; a.strideBias = strideBias;
  a.C = C; a.strideC = strideC; a.ldc = ldc; a.col_off = col_off;
  a.rows = rows; a.N = N; a.K = K; a.act = act; a.groups = groups;
  return launch_gemm(EPI_BIAS_ACT, a, (hipStream_t)stream);
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
  a.rows = rows; a.N = amx::round_up(n_valid, BN); a.K = K; a.groups = groups;
  a.n_valid = n_valid;
  const int S = ctx->S, Ad = ctx->A;
  a.shift = ctx->d_norm + 2 * S + 2 * Ad;  // mu_d
  a.scale = ctx->d_norm + 3 * S + 2 * Ad;  // sd_d
  return launch_gemm(EPI_UNNORM, a, (hipStream_t)stream);
}

extern "C" int amx_rff_features(amx_ctx* ctx, int rows, int n_valid, int F, int K, const float* x, int ldx,
                                const float* W, int ldw, const float* b, float scale, float* phi, int ldphi,
                                double* col_partials, const uint8_t* row_mask, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_rff_features: null ctx");
  int rc = check_common("amx_rff_features", 1, rows, K, x, ldx, W, ldw);
  if (rc) return rc;
  AMX_CHECK_ARG(F > 0 && F % BN == 0, "amx_rff_features: F=%d must be a multiple of %d", F, BN);
  AMX_CHECK_ARG(b && phi && col_partials && ldphi >= F, "amx_rff_features: null b/phi/partials or ldphi");
  AMX_CHECK_ARG(n_valid >= 0 && n_valid <= rows, "amx_rff_features: n_valid=%d rows=%d", n_valid, rows);
  GemmArgs a = {};
  a.A = x; a.lda = ldx;
  a.W = W; a.ldw = ldw;
  a.bias = b;
  a.C = phi; a.ldc = ldphi;
  a.rows = rows; a.N = F; a.K = K; a.groups = 1;
  a.n_valid = n_valid; a.rff_scale = scale; a.col_partials = col_partials; a.row_mask = row_mask;
  return launch_gemm(EPI_RFF, a, (hipStream_t)stream);
}
