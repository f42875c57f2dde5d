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

  // staging map: float4 index q = t + 256*j (j < 4) -> row q>>3, column 4*(q&7)
  const int st_r = t >> 3, st_c = (t & 7) * 4;

  float4 ra[4], rw[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = st_r + 32 * j;
      ra[j] = *reinterpret_cast<const float4*>(Ag + (long long)r * a.lda + k0 + st_c);
      rw[j] = *reinterpret_cast<const float4*>(Wg + (long long)r * a.ldw + k0 + st_c);
    }
  };
  auto lstore = [&](int buf) {
    float* As = smem + buf * TILE_FLOATS;
    float* Ws = As + BM * LDS_LD;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = st_r + 32 * j;
      *reinterpret_cast<float4*>(As + r * LDS_LD + st_c) = ra[j];
      *reinterpret_cast<float4*>(Ws + r * LDS_LD + st_c) = rw[j];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = a.K / BK;
  gload(0);
  lstore(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);

    const float* As = smem + cur * TILE_FLOATS;
    const float* Ws = As + BM * LDS_LD;
    float4 fa[2][4], fb[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        fa[m][v] = *reinterpret_cast<const float4*>(As + (wm * 64 + m * 32 + li) * LDS_LD + lh * 16 + v * 4);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        fb[n][v] = *reinterpret_cast<const float4*>(Ws + (wn * 64 + n * 32 + li) * LDS_LD + lh * 16 + v * 4);

#pragma unroll
    for (int v = 0; v < 4; ++v) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a0 = fa[0][v][e], a1 = fa[1][v][e];
        const float b0 = fb[0][v][e], b1 = fb[1][v][e];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

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
    // column sums of this wave's 64 rows -> LDS -> ordered sum of the two M-waves
    double* red = reinterpret_cast<double*>(smem);  // [2 (wm)][128 cols], reuses stage LDS
    float* Cg = a.C;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int col = col0 + n * 32 + li;
      const float bv = a.bias[col];
      double csum = 0.0;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = row0 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          const float z = acc[m][n][e] + bv;
          const float phi = cosf(z) * a.rff_scale;
          Cg[(long long)row * a.ldc + col] = phi;
          const bool valid = row < a.n_valid && (a.row_mask == nullptr || a.row_mask[row] != 0);
          csum += valid ? (double)phi : 0.0;
        }
      }
      csum += __shfl_xor(csum, 32);
      if (lh == 0) red[wm * BN + wn * 64 + n * 32 + li] = csum;
    }
    __syncthreads();
    if (t < BN) {
      const double s = red[t] + red[BN + t];
      a.col_partials[(long long)tm * a.N + tn * BN + t] = s;
    }
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
