// Per-lane kernels of the batched SimEnv step (gym-simenv/gym_simenv/envs/sim_env.py):
// state assembly, fp64 state update + fall/horizon termination + ensemble disagreement,
// masked resets from a device reset-state table, and the device Gaussian-MLP policy.
//
// These kernels are HBM/latency-bound per lane row (a few KB per lane); the layout is one
// wave64 per lane with lanes of the wave striding the state vector, so every row access
// is coalesced and every per-lane reduction is a wave reduction (no LDS).
//
// Numerics: the file is built with -ffp-contract=off.  Every expression below that the
// reference evaluates as separate IEEE operations (normalisation, state update,
// termination sums/products) must round exactly as numpy/torch-CPU do; termination is
// bit-exact by construction.
#include "amx_common.h"

namespace {

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---- assemble -----------------------------------------------------------------------
// x0 = [(s - mu_s)/sd_s, (a - mu_a)/sd_a, 0...] into every model's activation row.
// One wave per lane row; writes k0_pad columns for each of M models.
template <typename T>
__global__ __launch_bounds__(256) void k_assemble(const T* __restrict__ ob, const T* __restrict__ act,
                                                  const float* __restrict__ norm, float* __restrict__ buf,
                                                  long long stride_m, int ldk, int S, int A, int M, int k0_pad,
                                                  int B) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* mu_s = norm;
  const float* sd_s = norm + S;
  const float* mu_a = norm + 2 * S;
  const float* sd_a = norm + 2 * S + A;
  for (int j = lane; j < k0_pad; j += 64) {
    float x = 0.f;
    if (j < S) {
      const float s = (float)ob[(long long)b * S + j];
      x = (s - mu_s[j]) / sd_s[j];
    } else if (j < S + A) {
      const int k = j - S;
      const float v = (float)act[(long long)b * A + k];
      x = (v - mu_a[k]) / sd_a[k];
    }
    for (int m = 0; m < M; ++m) buf[m * stride_m + (long long)b * ldk + j] = x;
  }
}

// ---- disagreement ---------------------------------------------------------------------
// d = max over pairs (i<j) of ||p_i - p_j||_2: the pair differences are formed in fp32 as
// torch does (preds[i] - preds[j]), squared and summed in fp64, sqrt in fp64, rounded.
template <int MM>
__device__ inline float lane_disagreement(const float* __restrict__ preds, long long strideP, int ldp, int b,
                                          int S, int lane) {
  constexpr int NP = MM * (MM - 1) / 2;
  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;
  for (int j = lane; j < S; j += 64) {
    float v[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) v[m] = preds[m * strideP + (long long)b * ldp + j];
    int p = 0;
#pragma unroll
    for (int i = 0; i < MM; ++i)
#pragma unroll
      for (int k = i + 1; k < MM; ++k) {
        const float d = v[i] - v[k];
        acc[p++] += (double)d * (double)d;
      }
  }
  float best = 0.f;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float n = (float)sqrt(wave_sum(acc[p]));
    best = (p == 0 || n > best) ? n : best;
  }
  return best;
}

__device__ inline float disagreement_dispatch(int M, const float* preds, long long strideP, int ldp, int b, int S,
                                              int lane) {
  switch (M) {
    case 2: return lane_disagreement<2>(preds, strideP, ldp, b, S, lane);
    case 3: return lane_disagreement<3>(preds, strideP, ldp, b, S, lane);
    case 4: return lane_disagreement<4>(preds, strideP, ldp, b, S, lane);
    case 5: return lane_disagreement<5>(preds, strideP, ldp, b, S, lane);
    case 6: return lane_disagreement<6>(preds, strideP, ldp, b, S, lane);
    case 7: return lane_disagreement<7>(preds, strideP, ldp, b, S, lane);
    case 8: return lane_disagreement<8>(preds, strideP, ldp, b, S, lane);
    default: return 0.f;  // a single model has no pairs: torch max over an empty dim errors;
                          // the host refuses M == 1 for disagreement.
  }
}

__global__ __launch_bounds__(256) void k_disagreement(const float* __restrict__ preds, long long strideP, int ldp,
                                                      float* __restrict__ disc, int S, int M, int B) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float d = disagreement_dispatch(M, preds, strideP, ldp, b, S, lane);
  if (lane == 0) disc[b] = d;
}

// ---- step + termination -----------------------------------------------------------------
struct StepArgs {
  const float* preds; long long strideP; int ldp;
  const int32_t* model_idx;
  const double* ob; double* ob_next;
  int32_t* num_steps; uint8_t* done; float* disc;
  float* cost_in; int ldc;
  uint8_t* nonfinite;
  int S, M, B;
  amx_termination term;
};

__global__ __launch_bounds__(256) void k_step(StepArgs a) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= a.B) return;
  const amx_termination& T = a.term;
  const int S = a.S;
  const int k = a.model_idx[b];
  const float* pk = a.preds + (long long)k * a.strideP + (long long)b * a.ldp;
  const double* ob = a.ob + (long long)b * S;
  double* on = a.ob_next + (long long)b * S;

  // sim_env.py:158  ob += state_diff (float32 -> float64), then the in-place velocity
  // rescale of check_velocity (:264-267) when RecordVelAsPos and the check are enabled.
  const bool vscale = T.vel_check && T.record_vel_as_pos;
  bool vel_bad = false, bad = false;
  for (int j = lane; j < S; j += 64) {
    double x = ob[j] + (double)pk[j];
    if (vscale && j >= T.vel_offset) x = x / T.sampling_rate;
    on[j] = x;
    if (T.vel_check && j >= T.vel_offset) vel_bad |= fabs(x) > T.vel_thresh;
    bad |= !isfinite(x);
    if (a.cost_in) {
      a.cost_in[(long long)b * a.ldc + j] = (float)ob[j];
      a.cost_in[(long long)b * a.ldc + S + j] = (float)x;
    }
  }
  if (a.cost_in) {  // zero the K padding of the cost-input row
    for (int j = 2 * S + lane; j < a.ldc; j += 64) a.cost_in[(long long)b * a.ldc + j] = 0.f;
  }

  // fall check (sim_env.py:175-257): lane i < n evaluates body i from recomputed values
  // (identical fp64 ops as the stores above, so the same bits).
  bool hit = false;
  if (lane < T.n) {
    const int i = lane;
    auto val = [&](int j) {
      double x = ob[j] + (double)pk[j];
      if (vscale && j >= T.vel_offset) x = x / T.sampling_rate;
      return x;
    };
    if (T.shape[i] == AMX_SHAPE_SPHERE || T.shape[i] == AMX_SHAPE_CAPSULE) {
      double y;
      if (T.list_index_world[i]) {
        y = val(T.y_index[i]);
      } else {
        y = val(0) + val(T.y_index[i]);
      }
      if (T.shape[i] == AMX_SHAPE_SPHERE) {
        hit = y <= T.thresh[i];
      } else {
        const double ny = val(T.ny_index[i]);
        const double top = T.half_h[i] * ny;
        const double bot = T.neg_half_h[i] * ny;
        const double ytop = y + top;
        const double ybot = y + bot;
        hit = (ytop <= T.thresh[i]) || (ybot <= T.thresh[i]);
      }
    }  // box: check_box always False (sim_env.py:238-244)
  }
  const bool collided = __ballot(hit) != 0ull;
  const bool vexp = __ballot(vel_bad) != 0ull;
  const bool nf = __ballot(bad) != 0ull;

  float d = 0.f;
  if (a.disc) d = disagreement_dispatch(a.M, a.preds, a.strideP, a.ldp, b, S, lane);

  if (lane == 0) {
    const int ns = a.num_steps[b] + 1;  // sim_env.py:153
    a.num_steps[b] = ns;
    const bool horizon_done = ns >= T.horizon;  // :170
    a.done[b] = (horizon_done || collided || vexp) ? 1 : 0;
    if (a.disc) a.disc[b] = d;
    if (a.nonfinite) a.nonfinite[b] = nf ? 1 : 0;
  }
}

// ---- reset ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_reset(const uint8_t* __restrict__ mask, const double* __restrict__ table,
                                               int R, const int32_t* __restrict__ rows, uint32_t k0, uint32_t k1,
                                               const double* ob_src, double* ob_out, int32_t* num_steps,
                                               int32_t* model_idx, int32_t* reset_count, int32_t* row_out, int S,
                                               int M, int B) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const bool do_reset = (mask == nullptr) || mask[b] != 0;
  if (!do_reset) {
    if (ob_src != ob_out)
      for (int j = lane; j < S; j += 64) ob_out[(long long)b * S + j] = ob_src[(long long)b * S + j];
    if (lane == 0 && row_out) row_out[b] = -1;
    return;
  }
  const int rc = reset_count[b] + 1;  // sim_env.py:282: counter advances on every reset
  int row;
  if (rows) {
    row = rows[b];
  } else {
    const amx::u32x4 r = amx::philox4x32_10({(uint32_t)b, (uint32_t)rc, 0u, amx::kTagReset}, k0, k1);
    const uint64_t x = ((uint64_t)r.y << 32) | r.x;
    row = (int)(x % (uint64_t)R);
  }
  const double* src = table + (long long)row * S;
  for (int j = lane; j < S; j += 64) ob_out[(long long)b * S + j] = src[j];
  if (lane == 0) {
    reset_count[b] = rc;
    model_idx[b] = rc % M;  // :282-283
    num_steps[b] = 0;       // :277
    if (row_out) row_out[b] = row;
  }
}

// ---- policy ----------------------------------------------------------------------------------
// One workgroup = 256 threads = 16 lanes x 16 threads; every thread owns hidden units
// u = t16, t16+16, ...  Layer inputs are staged in LDS per lane.
constexpr int POL_LANES = 16;
constexpr int POL_MAXH = 256;

__global__ __launch_bounds__(256) void k_policy(const double* __restrict__ ob, const float* __restrict__ W1,
                                                const float* __restrict__ b1, int H1, const float* __restrict__ W2,
                                                const float* __restrict__ b2, int H2, const float* __restrict__ W3,
                                                const float* __restrict__ b3, const double* __restrict__ nscale,
                                                const double* __restrict__ noise, uint32_t k0, uint32_t k1,
                                                uint32_t ctr_lo, uint32_t ctr_hi, int eval_mode,
                                                double* __restrict__ act, float* __restrict__ mean_out, int S,
                                                int A, int B) {
  extern __shared__ __attribute__((aligned(16))) float psm[];
  // [POL_LANES][S] observations, then [POL_LANES][H1] and [POL_LANES][H2]
  float* so = psm;
  float* sh1 = so + POL_LANES * S;
  float* sh2 = sh1 + POL_LANES * H1;
  const int t = threadIdx.x;
  const int lb = t >> 4, u0 = t & 15;
  const int b0 = blockIdx.x * POL_LANES;
  for (int i = t; i < POL_LANES * S; i += 256) {
    const int l = i / S, j = i - l * S;
    const int b = b0 + l;
    so[i] = (b < B) ? (float)ob[(long long)b * S + j] : 0.f;  // np.float32(observation)
  }
  __syncthreads();
  const int b = b0 + lb;
  for (int u = u0; u < H1; u += 16) {
    float s = 0.f;
    const float* w = W1 + (long long)u * S;
    for (int j = 0; j < S; ++j) s = fmaf(w[j], so[lb * S + j], s);
    sh1[lb * H1 + u] = tanhf(s + b1[u]);
  }
  __syncthreads();
  for (int u = u0; u < H2; u += 16) {
    float s = 0.f;
    const float* w = W2 + (long long)u * H1;
    for (int j = 0; j < H1; ++j) s = fmaf(w[j], sh1[lb * H1 + j], s);
    sh2[lb * H2 + u] = tanhf(s + b2[u]);
  }
  __syncthreads();
  if (b >= B) return;
  for (int u = u0; u < A; u += 16) {
    float s = 0.f;
    const float* w = W3 + (long long)u * H2;
    for (int j = 0; j < H2; ++j) s = fmaf(w[j], sh2[lb * H2 + j], s);
    const float m = s + b3[u];  // FCNetwork out_scale = 1, out_shift = 0 (fc_network.py:54)
    if (mean_out) mean_out[(long long)b * A + u] = m;
    double a_out;
    if (eval_mode) {
      a_out = (double)m;
    } else {
      double n;
      if (noise) {
        n = noise[(long long)b * A + u];
      } else {
        // Box-Muller on one Philox block: pair p = u/2 yields normals for u = 2p, 2p+1
        const int p = u >> 1;
        const amx::u32x4 r =
            amx::philox4x32_10({(uint32_t)b, ctr_lo, ((uint32_t)p << 8) | (ctr_hi & 0xffu), amx::kTagPolicy}, k0, k1);
        const double u1 = 1.0 - amx::u53(r.x, r.y);  // (0, 1]
        const double u2 = amx::u53(r.z, r.w);
        const double rad = sqrt(-2.0 * log(u1));
        const double ang = 6.283185307179586 * u2;
        n = (u & 1) ? rad * sin(ang) : rad * cos(ang);
      }
      a_out = (double)m + nscale[u] * n;  // gaussian_mlp.py:102-103 (float32 + float64)
    }
    act[(long long)b * A + u] = a_out;
  }
}

__global__ void k_philox(uint32_t k0, uint32_t k1, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const amx::u32x4 r = amx::philox4x32_10({(uint32_t)i, c1, c2, c3}, k0, k1);
  out[4 * i + 0] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

inline dim3 lanes_grid(int B) { return dim3((unsigned)((B + 3) / 4)); }  // 4 lane-waves per block

}  // namespace

extern "C" int amx_assemble_input(amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                                  long long stride_m, int ldk, int B, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "amx_assemble_input: context has no normalizers");
  AMX_CHECK_ARG(ob && act && act_buf, "amx_assemble_input: null pointer");
  AMX_CHECK_ARG(B >= 0, "amx_assemble_input: B=%d", B);
  AMX_CHECK_ARG(ldk >= ctx->k0_pad, "amx_assemble_input: ldk=%d < k0_pad=%d", ldk, ctx->k0_pad);
  AMX_CHECK_ARG(ctx->M == 1 || stride_m >= (long long)ldk * B, "amx_assemble_input: stride_m too small");
  if (B == 0) return AMX_OK;
  hipStream_t s = (hipStream_t)stream;
  if (in_dtype == AMX_IN_F64) {
    hipLaunchKernelGGL(k_assemble<double>, lanes_grid(B), dim3(256), 0, s, (const double*)ob, (const double*)act,
                       ctx->d_norm, act_buf, stride_m, ldk, ctx->S, ctx->A, ctx->M, ctx->k0_pad, B);
  } else if (in_dtype == AMX_IN_F32) {
    hipLaunchKernelGGL(k_assemble<float>, lanes_grid(B), dim3(256), 0, s, (const float*)ob, (const float*)act,
                       ctx->d_norm, act_buf, stride_m, ldk, ctx->S, ctx->A, ctx->M, ctx->k0_pad, B);
  } else {
    AMX_CHECK_ARG(false, "amx_assemble_input: in_dtype=%d", in_dtype);
  }
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_step(amx_ctx* ctx, const float* preds, int ldp, long long strideP, const int32_t* model_idx,
                        const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                        float* cost_in, int ldc, uint8_t* nonfinite, int B, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_term, "amx_step: context has no termination config");
  AMX_CHECK_ARG(preds && model_idx && ob && ob_next && num_steps && done, "amx_step: null pointer");
  AMX_CHECK_ARG(ldp >= ctx->S && B >= 0, "amx_step: ldp=%d B=%d", ldp, B);
  AMX_CHECK_ARG(!disc || ctx->M >= 2, "amx_step: disagreement needs >= 2 models");
  AMX_CHECK_ARG(!cost_in || ldc >= 2 * ctx->S, "amx_step: ldc=%d < 2S", ldc);
  AMX_CHECK_ARG(ob != ob_next, "amx_step: ob and ob_next must not alias");
  if (B == 0) return AMX_OK;
  StepArgs a;
  a.preds = preds; a.strideP = strideP; a.ldp = ldp;
  a.model_idx = model_idx; a.ob = ob; a.ob_next = ob_next;
  a.num_steps = num_steps; a.done = done; a.disc = disc;
  a.cost_in = cost_in; a.ldc = ldc; a.nonfinite = nonfinite;
  a.S = ctx->S; a.M = ctx->M; a.B = B; a.term = ctx->term;
  hipLaunchKernelGGL(k_step, lanes_grid(B), dim3(256), 0, (hipStream_t)stream, a);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_disagreement(amx_ctx* ctx, const float* preds, int ldp, long long strideP, float* disc, int B,
                                void* stream) {
  AMX_CHECK_ARG(ctx && preds && disc, "amx_disagreement: null pointer");
  AMX_CHECK_ARG(ctx->M >= 2, "amx_disagreement: needs >= 2 models (M=%d)", ctx->M);
  AMX_CHECK_ARG(ldp >= ctx->S && B >= 0, "amx_disagreement: ldp=%d B=%d", ldp, B);
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_disagreement, lanes_grid(B), dim3(256), 0, (hipStream_t)stream, preds, strideP, ldp, disc,
                     ctx->S, ctx->M, B);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_reset_lanes(amx_ctx* ctx, const uint8_t* mask, const double* table, int R, const int32_t* rows,
                               uint64_t seed, const double* ob_src, double* ob_out, int32_t* num_steps,
                               int32_t* model_idx, int32_t* reset_count, int32_t* row_out, int B, void* stream) {
  AMX_CHECK_ARG(ctx && table && ob_out && num_steps && model_idx && reset_count, "amx_reset_lanes: null pointer");
  AMX_CHECK_ARG(R > 0 && B >= 0, "amx_reset_lanes: R=%d B=%d", R, B);
  AMX_CHECK_ARG(mask == nullptr || ob_src != nullptr, "amx_reset_lanes: masked reset needs ob_src");
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_reset, lanes_grid(B), dim3(256), 0, (hipStream_t)stream, mask, table, R, rows,
                     (uint32_t)seed, (uint32_t)(seed >> 32), ob_src, ob_out, num_steps, model_idx, reset_count,
                     row_out, ctx->S, ctx->M, B);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_policy_act(amx_ctx* ctx, const double* ob, int B, const float* W1, const float* b1, int H1,
                              const float* W2, const float* b2, int H2, const float* W3, const float* b3,
                              const double* noise_scale, const double* noise, uint64_t seed, uint64_t counter,
                              int eval_mode, double* act, float* mean, void* stream) {
  AMX_CHECK_ARG(ctx && ob && W1 && b1 && W2 && b2 && W3 && b3 && act, "amx_policy_act: null pointer");
  AMX_CHECK_ARG(eval_mode || noise_scale, "amx_policy_act: noise_scale required unless eval_mode");
  AMX_CHECK_ARG(H1 > 0 && H1 <= POL_MAXH && H2 > 0 && H2 <= POL_MAXH, "amx_policy_act: H1=%d H2=%d", H1, H2);
  AMX_CHECK_ARG(B >= 0, "amx_policy_act: B=%d", B);
  if (B == 0) return AMX_OK;
  const size_t lds = sizeof(float) * POL_LANES * (ctx->S + H1 + H2);
  AMX_CHECK_ARG(lds <= 160 * 1024, "amx_policy_act: S too large for LDS staging");
  dim3 grid((B + POL_LANES - 1) / POL_LANES);
  hipLaunchKernelGGL(k_policy, grid, dim3(256), lds, (hipStream_t)stream, ob, W1, b1, H1, W2, b2, H2, W3, b3,
                     noise_scale, noise, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)counter,
                     (uint32_t)(counter >> 32), eval_mode, act, mean, ctx->S, ctx->A, B);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_philox(amx_ctx* ctx, uint64_t seed, uint32_t ctr1, uint32_t ctr2, uint32_t ctr3, uint32_t* out,
                          int n, void* stream) {
  AMX_CHECK_ARG(ctx && out && n >= 0, "amx_philox: bad argument");
  if (n == 0) return AMX_OK;
  hipLaunchKernelGGL(k_philox, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (uint32_t)seed,
                     (uint32_t)(seed >> 32), ctr1, ctr2, ctr3, out, n);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
