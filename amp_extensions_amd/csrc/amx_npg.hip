// The NPG policy update on the device: the learner step that consumes the rollout in the
// reference's MILO loop (mjrl NPG.train_from_paths, mjrl/mjrl/algos/npg_cg.py:113-199).
//
// Policy: mjrl MLP (gaussian_mlp.py:7-155) — mean = W3 tanh(W2 tanh(W1 x + b1) + b2) + b3,
// a ~ N(mean, exp(log_std)^2); parameters packed in the reference's flat order
// (trainable_params: W1 [H1][S], b1, W2 [H2][H1], b2, W3 [A][H2], b3, log_std [A]).
//
// One pass kernel, three modes, each block owning a contiguous run of rows and writing one
// fp64 partial vector (fixed-order reduction afterwards: deterministic):
//   VPG  grad of mean(LR * adv) at new == old (batch_reinforce.py:58-62, npg_cg.py:66-86):
//        dmean = adv/N * z/sigma, dlog_std = adv/N * (z^2 - 1), z = (a - mean)/sigma;
//   FVP  the mean-parameter part of NPG.HVP (npg_cg.py:87-106): the Hessian of mean_kl
//        (gaussian_mlp.py:144-155) at new == old is J^T diag(2/(2 sigma^2 + 1e-8)) J / N for
//        the mean network; the JVP J v is propagated forward, then back-propagated (the
//        log_std block, a diagonal constant, and the damping are added by the caller);
//   EVAL mean(LR * adv) and mean_kl of new vs old parameters (surr_after, kl_old_new,
//        npg_cg.py:181-183).
// Rows are processed in chunks of 32 staged in LDS with the weights; every thread owns a
// fixed set of gradient entries and accumulates its chunk sums in fp64 registers.
// Hidden widths are fixed at 32 (MILO's actor_model_hidden, milo/milo/arguments.py:95).
#include "amx_common.h"

namespace {

constexpr int NH = 32;     // hidden width (both layers)
constexpr int RC = 32;     // rows per chunk
constexpr int NT = 256;    // threads per block
constexpr int MAXS = 256;  // max state dim
constexpr int MAXA = 64;   // max action dim
constexpr int HP = NH + 1; // padded row of the [RC][NH] activation tiles

enum { NPG_VPG = 0, NPG_FVP = 1, NPG_EVAL = 2 };

struct NpgArgs {
  int mode, N, S, A, SP;     // SP: odd LDS row stride of W1 / X (conflict-free column reads)
  int rows_per_block;
  const void* obs; int obs_f64; long long ldo;
  const void* act; int act_f64; long long lda;
  const double* adv;         // VPG / EVAL (whitened advantages)
  const float* theta;        // packed parameters (old, for EVAL)
  const float* vec;          // FVP: tangent; EVAL: new parameters
  double* partials;          // VPG/FVP: [blocks][P]; EVAL: [blocks][2]
  int P;
};

struct Lay {  // offsets into the packed parameter vector
  int w1, b1, w2, b2, w3, b3, ls;
  __device__ Lay(int S, int A) {
    w1 = 0; b1 = NH * S; w2 = b1 + NH; b2 = w2 + NH * NH; w3 = b2 + NH; b3 = w3 + A * NH; ls = b3 + A;
  }
};

// LDS image of one parameter set: W1 [NH][SP], b1, W2 [NH][HP], b2, W3 [A][HP], b3, ls
struct PSet {
  float *w1, *b1, *w2, *b2, *w3, *b3, *ls;
};

__device__ inline float* carve(float*& p, int n) {
  float* r = p;
  p += (n + 3) & ~3;
  return r;
}

__device__ inline void load_params(const float* __restrict__ src, const Lay& L, int S, int A, int SP, PSet& d) {
  for (int e = threadIdx.x; e < NH * S; e += NT) d.w1[(e / S) * SP + e % S] = src[L.w1 + e];
  for (int e = threadIdx.x; e < NH * NH; e += NT) d.w2[(e / NH) * HP + e % NH] = src[L.w2 + e];
  for (int e = threadIdx.x; e < A * NH; e += NT) d.w3[(e / NH) * HP + e % NH] = src[L.w3 + e];
  for (int e = threadIdx.x; e < NH; e += NT) {
    d.b1[e] = src[L.b1 + e];
    d.b2[e] = src[L.b2 + e];
  }
  for (int e = threadIdx.x; e < A; e += NT) {
    d.b3[e] = src[L.b3 + e];
    d.ls[e] = src[L.ls + e];
  }
}

// out[r][j] = act(b[j] + sum_k W[j][k] in[r][k]) for r < RC, j < NH; thread: j = t&31,
// rows rg + 8q.  in row stride ldi, W row stride ldw.  Returns the pre-activation sums via
// the callback order used by the caller.
__device__ inline void dense_nh(const float* W, int ldw, const float* b, const float* in, int ldi, int K, float (&acc)[4]) {
  const int j = threadIdx.x & 31, rg = threadIdx.x >> 5;
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = b ? b[j] : 0.f;
  for (int k = 0; k < K; ++k) {
    const float w = W[j * ldw + k];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = fmaf(w, in[(rg + 8 * q) * ldi + k], acc[q]);
  }
}

__global__ __launch_bounds__(NT, 1) void k_npg(NpgArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int S = a.S, A = a.A, SP = a.SP, t = threadIdx.x;
  const Lay L(S, A);
  float* p = sm;
  PSet th, tv;
  th.w1 = carve(p, NH * SP); th.b1 = carve(p, NH); th.w2 = carve(p, NH * HP); th.b2 = carve(p, NH);
  th.w3 = carve(p, A * HP); th.b3 = carve(p, A); th.ls = carve(p, A);
  const bool two = a.mode != NPG_VPG;
  if (two) {
    tv.w1 = carve(p, NH * SP); tv.b1 = carve(p, NH); tv.w2 = carve(p, NH * HP); tv.b2 = carve(p, NH);
    tv.w3 = carve(p, A * HP); tv.b3 = carve(p, A); tv.ls = carve(p, A);
  }
  float* X = carve(p, RC * SP);
  float* H1 = carve(p, RC * HP);
  float* H2 = carve(p, RC * HP);
  float* D1 = carve(p, RC * HP);   // FVP: JVP of layer 1, then the backward delta
  float* D2 = carve(p, RC * HP);
  float* G = carve(p, RC * MAXA);  // output-layer gradient (or, EVAL: new mean)
  float* M = carve(p, RC * MAXA);  // mean (or JVP of the mean)
  double* red = reinterpret_cast<double*>(carve(p, 2 * 2 * NT));

  load_params(a.theta, L, S, A, SP, th);
  if (two) load_params(a.vec, L, S, A, SP, tv);

  // gradient accumulators owned by this thread (fp64)
  double gw1[MAXS / 8], gw2[NH * NH / NT], gw3[MAXA * NH / NT], gb = 0.0;
#pragma unroll
  for (int m = 0; m < MAXS / 8; ++m) gw1[m] = 0.0;
#pragma unroll
  for (int m = 0; m < NH * NH / NT; ++m) gw2[m] = 0.0;
#pragma unroll
  for (int m = 0; m < MAXA * NH / NT; ++m) gw3[m] = 0.0;
  double ev_surr = 0.0, ev_kl = 0.0;
  const double invN = 1.0 / (double)a.N;

  const int r0 = blockIdx.x * a.rows_per_block;
  const int r1 = min(a.N, r0 + a.rows_per_block);
  for (int c0 = r0; c0 < r1; c0 += RC) {
    const int nr = min(RC, r1 - c0);
    __syncthreads();  // previous chunk's tiles are consumed (and the parameters are loaded)
    for (int e = t; e < RC * S; e += NT) {
      const int r = e / S, k = e % S;
      float v = 0.f;
      if (r < nr) {
        const long long off = (long long)(c0 + r) * a.ldo + k;
        v = a.obs_f64 ? (float)static_cast<const double*>(a.obs)[off] : static_cast<const float*>(a.obs)[off];
      }
      X[r * SP + k] = v;
    }
    __syncthreads();
    // ---- forward (and, FVP, the tangent) of the two tanh layers --------------------------
    const int j = t & 31, rg = t >> 5;
    float acc[4], dac[4];
    dense_nh(th.w1, SP, th.b1, X, SP, S, acc);
    if (a.mode == NPG_FVP) dense_nh(tv.w1, SP, tv.b1, X, SP, S, dac);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float h = tanhf(acc[q]);
      H1[(rg + 8 * q) * HP + j] = h;
      if (a.mode == NPG_FVP) D1[(rg + 8 * q) * HP + j] = dac[q] * (1.f - h * h);
    }
    if (a.mode == NPG_EVAL) {  // second forward with the new parameters into D1
      dense_nh(tv.w1, SP, tv.b1, X, SP, S, dac);
#pragma unroll
      for (int q = 0; q < 4; ++q) D1[(rg + 8 * q) * HP + j] = tanhf(dac[q]);
    }
    __syncthreads();
    dense_nh(th.w2, HP, th.b2, H1, HP, NH, acc);
    if (a.mode == NPG_FVP) {
      float d2[4], d3[4];
      dense_nh(tv.w2, HP, tv.b2, H1, HP, NH, d2);     // vW2 h1 + vb2
      dense_nh(th.w2, HP, nullptr, D1, HP, NH, d3);   // W2 dh1
#pragma unroll
      for (int q = 0; q < 4; ++q) dac[q] = d2[q] + d3[q];
    } else if (a.mode == NPG_EVAL) {
      dense_nh(tv.w2, HP, tv.b2, D1, HP, NH, dac);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float h = tanhf(acc[q]);
      H2[(rg + 8 * q) * HP + j] = h;
      if (a.mode == NPG_FVP) D2[(rg + 8 * q) * HP + j] = dac[q] * (1.f - h * h);
      if (a.mode == NPG_EVAL) D2[(rg + 8 * q) * HP + j] = tanhf(dac[q]);
    }
    __syncthreads();
    // ---- output layer: mean (M); FVP: JVP of the mean (M); EVAL: new mean (G) ---------------
    for (int e = t; e < RC * A; e += NT) {
      const int r = e / A, d = e % A;
      float m = th.b3[d];
      for (int k = 0; k < NH; ++k) m = fmaf(th.w3[d * HP + k], H2[r * HP + k], m);
      if (a.mode == NPG_FVP) {
        float v1 = tv.b3[d], v2 = 0.f;
        for (int k = 0; k < NH; ++k) v1 = fmaf(tv.w3[d * HP + k], H2[r * HP + k], v1);
        for (int k = 0; k < NH; ++k) v2 = fmaf(th.w3[d * HP + k], D2[r * HP + k], v2);
        m = v1 + v2;
      } else if (a.mode == NPG_EVAL) {
        float mn = tv.b3[d];
        for (int k = 0; k < NH; ++k) mn = fmaf(tv.w3[d * HP + k], D2[r * HP + k], mn);
        G[r * MAXA + d] = mn;
      }
      M[r * MAXA + d] = m;
    }
    __syncthreads();
    if (a.mode == NPG_EVAL) {
      // per row: LL_new - LL_old and sample_kl (gaussian_mlp.py:110-155), one thread per row
      if (t < nr) {
        const int r = t;
        const long long ro = (long long)(c0 + r);
        float dll = 0.f, kl = 0.f, sls_o = 0.f, sls_n = 0.f;
        for (int d = 0; d < A; ++d) {
          const float ac = a.act_f64 ? (float)static_cast<const double*>(a.act)[ro * a.lda + d]
                                     : static_cast<const float*>(a.act)[ro * a.lda + d];
          const float so = expf(th.ls[d]), sn = expf(tv.ls[d]);
          const float zo = (ac - M[r * MAXA + d]) / so, zn = (ac - G[r * MAXA + d]) / sn;
          dll += -0.5f * zn * zn - (-0.5f * zo * zo);
          sls_o += th.ls[d];
          sls_n += tv.ls[d];
          const float dm = M[r * MAXA + d] - G[r * MAXA + d];
          const float Nr = dm * dm + so * so - sn * sn, Dr = 2.f * sn * sn + 1e-8f;
          kl += Nr / Dr + tv.ls[d] - th.ls[d];
        }
        dll += -sls_n + sls_o;
        ev_surr += (double)(expf(dll) * (float)a.adv[ro]);
        ev_kl += (double)kl;
      }
      continue;
    }
    // ---- output-layer gradient G [RC][A] ---------------------------------------------------
    for (int e = t; e < RC * A; e += NT) {
      const int r = e / A, d = e % A;
      float g = 0.f;
      if (r < nr) {
        const float sd = expf(th.ls[d]);
        if (a.mode == NPG_VPG) {
          const long long ro = (long long)(c0 + r);
          const float ac = a.act_f64 ? (float)static_cast<const double*>(a.act)[ro * a.lda + d]
                                     : static_cast<const float*>(a.act)[ro * a.lda + d];
          const float z = (ac - M[r * MAXA + d]) / sd;
          g = (float)(a.adv[ro] * invN) * (z / sd);
        } else {
          const float c = 2.f / (2.f * sd * sd + 1e-8f);
          g = (float)((double)(M[r * MAXA + d] * c) * invN);
        }
      }
      G[r * MAXA + d] = g;
    }
    // log_std gradient (VPG): sum_r adv/N (z^2 - 1), threads [128, 128 + A)
    if (a.mode == NPG_VPG && t >= 128 && t < 128 + A) {
      const int d = t - 128;
      const float sd = expf(th.ls[d]);
      for (int r = 0; r < nr; ++r) {
        const long long ro = (long long)(c0 + r);
        const float ac = a.act_f64 ? (float)static_cast<const double*>(a.act)[ro * a.lda + d]
                                   : static_cast<const float*>(a.act)[ro * a.lda + d];
        const float z = (ac - M[r * MAXA + d]) / sd;
        gb += a.adv[ro] * invN * (double)(z * z - 1.f);
      }
    }
    __syncthreads();
    // ---- backward ------------------------------------------------------------------------
    // gW3[d][k] += sum_r G[r][d] H2[r][k]; entries e = t + NT*m (d = e>>5, k = e&31)
#pragma unroll
    for (int m = 0; m < MAXA * NH / NT; ++m) {
      const int e = t + NT * m, d = e >> 5, k = e & 31;
      if (d < A) {
        float s = 0.f;
        for (int r = 0; r < nr; ++r) s = fmaf(G[r * MAXA + d], H2[r * HP + k], s);
        gw3[m] += (double)s;
      }
    }
    if (t >= 64 && t < 64 + A) {  // gb3
      float s = 0.f;
      for (int r = 0; r < nr; ++r) s += G[r * MAXA + (t - 64)];
      gb += (double)s;
    }
    // D2[r][j] = (sum_d G[r][d] W3[d][j]) (1 - H2^2)
    {
      float s[4] = {0.f, 0.f, 0.f, 0.f};
      for (int d = 0; d < A; ++d) {
        const float w = th.w3[d * HP + j];
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] = fmaf(G[(rg + 8 * q) * MAXA + d], w, s[q]);
      }
      __syncthreads();  // D2 (JVP) was read by the output layer above
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float h = H2[(rg + 8 * q) * HP + j];
        D2[(rg + 8 * q) * HP + j] = s[q] * (1.f - h * h);
      }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < NH * NH / NT; ++m) {  // gW2[jj][i] += sum_r D2[r][jj] H1[r][i]
      const int e = t + NT * m, jj = e >> 5, i = e & 31;
      float s = 0.f;
      for (int r = 0; r < nr; ++r) s = fmaf(D2[r * HP + jj], H1[r * HP + i], s);
      gw2[m] += (double)s;
    }
    if (t >= 32 && t < 64) {  // gb2
      float s = 0.f;
      for (int r = 0; r < nr; ++r) s += D2[r * HP + (t - 32)];
      gb += (double)s;
    }
    {  // D1[r][i] = (sum_jj D2[r][jj] W2[jj][i]) (1 - H1^2)
      float s[4] = {0.f, 0.f, 0.f, 0.f};
      for (int jj = 0; jj < NH; ++jj) {
        const float w = th.w2[jj * HP + j];
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] = fmaf(D2[(rg + 8 * q) * HP + jj], w, s[q]);
      }
      __syncthreads();  // D1 (JVP) was read by layer 2 above
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float h = H1[(rg + 8 * q) * HP + j];
        D1[(rg + 8 * q) * HP + j] = s[q] * (1.f - h * h);
      }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MAXS / 8; ++m) {  // gW1[i][k] += sum_r D1[r][i] X[r][k], i = t&31, k = rg + 8m
      const int k = rg + 8 * m;
      if (k < S) {
        float s = 0.f;
        for (int r = 0; r < nr; ++r) s = fmaf(D1[r * HP + j], X[r * SP + k], s);
        gw1[m] += (double)s;
      }
    }
    if (t < 32) {  // gb1
      float s = 0.f;
      for (int r = 0; r < nr; ++r) s += D1[r * HP + t];
      gb += (double)s;
    }
  }

  if (a.mode == NPG_EVAL) {
    // block sums of (surr, kl) in fixed order
    red[t] = ev_surr;
    red[NT + t] = ev_kl;
    __syncthreads();
    if (t == 0) {
      double s0 = 0.0, s1 = 0.0;
      for (int i = 0; i < NT; ++i) {
        s0 += red[i];
        s1 += red[NT + i];
      }
      a.partials[2LL * blockIdx.x] = s0;
      a.partials[2LL * blockIdx.x + 1] = s1;
    }
    return;
  }
  double* out = a.partials + (long long)blockIdx.x * a.P;
  const int j = t & 31, rg = t >> 5;
#pragma unroll
  for (int m = 0; m < MAXS / 8; ++m) {
    const int k = rg + 8 * m;
    if (k < S) out[L.w1 + j * S + k] = gw1[m];
  }
#pragma unroll
  for (int m = 0; m < NH * NH / NT; ++m) out[L.w2 + t + NT * m] = gw2[m];
#pragma unroll
  for (int m = 0; m < MAXA * NH / NT; ++m) {
    const int e = t + NT * m;
    if ((e >> 5) < A) out[L.w3 + e] = gw3[m];
  }
  if (t < 32) out[L.b1 + t] = gb;
  else if (t < 64) out[L.b2 + t - 32] = gb;
  else if (t < 64 + A) out[L.b3 + t - 64] = gb;
  else if (t >= 128 && t < 128 + A) out[L.ls + t - 128] = a.mode == NPG_VPG ? gb : 0.0;
}

// out[c] = sum_b partials[b][c] in a fixed order (deterministic): stage 1 sums runs of RB
// consecutive blocks per column (grid.y = run), stage 2 sums the runs in order.
constexpr int RB = 16;
__global__ void k_npg_reduce1(const double* __restrict__ part, int nb, int P, double* __restrict__ mid) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P) return;
  const int b0 = blockIdx.y * RB, b1 = min(nb, b0 + RB);
  double s = 0.0;
  for (int b = b0; b < b1; ++b) s += part[(long long)b * P + c];
  mid[(long long)blockIdx.y * P + c] = s;
}
__global__ void k_npg_reduce2(const double* __restrict__ mid, int nr, int P, double* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P) return;
  double s = 0.0;
  for (int r = 0; r < nr; ++r) s += mid[(long long)r * P + c];
  out[c] = s;
}

size_t npg_lds_bytes(int S, int A, int mode) {
  const int SP = (S | 1);
  auto r4 = [](int n) { return (size_t)((n + 3) & ~3); };
  const size_t pset = r4(NH * SP) + r4(NH) + r4(NH * HP) + r4(NH) + r4(A * HP) + r4(A) + r4(A);
  return sizeof(float) * (pset * (mode == NPG_VPG ? 1 : 2) + r4(RC * SP) + 4 * r4(RC * HP) + 2 * r4(RC * MAXA) +
                          r4(4 * NT));
}

}  // namespace

extern "C" long long amx_npg_param_count(int S, int A) {
  return (long long)NH * S + NH + NH * NH + NH + (long long)A * NH + A + A;
}

extern "C" int amx_npg_pass(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo,
                            const void* act, int act_dtype, long long lda, const double* adv, const float* theta,
                            const float* vec, int rows_per_block, double* partials, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_npg_pass: null ctx");
  const int S = ctx->S, A = ctx->A;
  AMX_CHECK_ARG(mode >= NPG_VPG && mode <= NPG_EVAL, "amx_npg_pass: mode=%d", mode);
  AMX_CHECK_ARG(S > 0 && S <= MAXS && A > 0 && A <= MAXA, "amx_npg_pass: S=%d (<= %d), A=%d (<= %d)", S, MAXS, A,
                MAXA);
  AMX_CHECK_ARG(N > 0 && rows_per_block > 0 && rows_per_block % RC == 0,
                "amx_npg_pass: N=%d rows_per_block=%d (multiple of %d)", N, rows_per_block, RC);
  AMX_CHECK_ARG(obs && act && theta && partials, "amx_npg_pass: null buffer");
  AMX_CHECK_ARG((mode == NPG_FVP || adv) && (mode == NPG_VPG || vec), "amx_npg_pass: adv/vec missing for mode %d",
                mode);
  AMX_CHECK_ARG(ldo >= S && lda >= A, "amx_npg_pass: ldo=%lld lda=%lld", ldo, lda);
  NpgArgs a = {};
  a.mode = mode; a.N = N; a.S = S; a.A = A; a.SP = S | 1; a.rows_per_block = rows_per_block;
  a.obs = obs; a.obs_f64 = obs_dtype == AMX_IN_F64; a.ldo = ldo;
  a.act = act; a.act_f64 = act_dtype == AMX_IN_F64; a.lda = lda;
  a.adv = adv; a.theta = theta; a.vec = vec; a.partials = partials;
  a.P = (int)amx_npg_param_count(S, A);
  const size_t lds = npg_lds_bytes(S, A, mode);
  AMX_CHECK_ARG(lds <= 160 * 1024, "amx_npg_pass: %zu B of LDS", lds);
  const int blocks = (N + rows_per_block - 1) / rows_per_block;
  hipLaunchKernelGGL(k_npg, dim3(blocks), dim3(NT), lds, (hipStream_t)stream, a);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_reduce(amx_ctx* ctx, const double* partials, int blocks, int P, double* out, void* stream) {
  AMX_CHECK_ARG(ctx && partials && out && blocks > 0 && P > 0, "amx_npg_reduce: bad arguments");
  const int runs = (blocks + RB - 1) / RB;
  if (runs == 1) {
    hipLaunchKernelGGL(k_npg_reduce2, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, partials, blocks, P,
                       out);
    AMX_CHECK_LAUNCH();
    return AMX_OK;
  }
  // the runs' sums go to a context-owned scratch (grown on demand, freed with the context)
  const size_t need = sizeof(double) * (size_t)runs * P;
  if (ctx->npg_scratch_bytes < need) {
    if (ctx->d_npg_scratch) AMX_CHECK_HIP(hipFree(ctx->d_npg_scratch));
    ctx->d_npg_scratch = nullptr;
    ctx->npg_scratch_bytes = 0;
    if (hipMalloc((void**)&ctx->d_npg_scratch, need) != hipSuccess) {
      amx::set_error("amx_npg_reduce: hipMalloc of %zu B failed", need);
      return AMX_E_NOMEM;
    }
    ctx->npg_scratch_bytes = need;
  }
  hipLaunchKernelGGL(k_npg_reduce1, dim3((P + 255) / 256, runs), dim3(256), 0, (hipStream_t)stream, partials, blocks,
                     P, ctx->d_npg_scratch);
  AMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_npg_reduce2, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, ctx->d_npg_scratch,
                     runs, P, out);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
