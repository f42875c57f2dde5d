// Returns, value-baseline features / head and GAE over the rollout's trajectories: the
// consumer of the sampler output in the reference's NPG step (mjrl BatchREINFORCE.train_step,
// mjrl/mjrl/algos/batch_reinforce.py:176-180), kept on the device so the rollout buffers
// never round-trip through host path dicts.
//
// Trajectory layout ("segment grid", include/amx_hip.h): lane l owns rows
// r(t, l) = base[l] + t * stride for t < len[l]; end[r] marks trajectory ends.  Engine
// buffers map lanes to persistent SimEnv lanes (several trajectories per lane, separated by
// done flags); concatenated mjrl paths map one lane to one path.
//
// All fp64 algebra is written in the reference's evaluation order and compiled with
// -ffp-contract=off, so returns/advantages are bit-identical to numpy's for the same
// baseline values.
#include "amx_common.h"

namespace {

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

struct Grid {
  int T, L;
  const int32_t* len;
  const int64_t* base;
  long long stride;
  __device__ int length(int l) const { return len ? len[l] : T; }
  __device__ long long row(int t, int l) const { return (base ? base[l] : (long long)l) + (long long)t * stride; }
};

// MLPBaseline._features (mlp_baseline.py:36-59).  One wave per lane walks the lane's rows
// in time order (the in-trajectory position is a running counter reset after each end).
__global__ __launch_bounds__(256) void k_value_features(Grid g, const int32_t* __restrict__ t0,
                                                        const uint8_t* __restrict__ end,
                                                        const double* __restrict__ obs, int ldo, int S, int kf,
                                                        float* __restrict__ feat, int ldf) {
  const int l = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (l >= g.L) return;
  const int n = g.length(l);
  int tpos = t0 ? t0[l] : 0;
  for (int t = 0; t < n; ++t) {
    const long long r = g.row(t, l);
    const double* o = obs + r * ldo;
    float* f = feat + r * ldf;
    for (int j = lane; j < kf; j += 64) {
      float v = 0.f;
      if (j < S) {
        double x = o[j];
        x = x < -10.0 ? -10.0 : (x > 10.0 ? 10.0 : x);  // np.clip (NaN passes through)
        v = (float)(x / 10.0);
      } else if (j < S + 4) {
        const double al = (double)tpos / 1000.0;         // np.arange(l) / 1000.0
        const int e = j - S + 1;                         // al ** (j+1)
        const double p = e == 1 ? al : (e == 2 ? al * al : pow(al, (double)e));
        v = (float)p;
      }
      f[j] = v;
    }
    tpos = end[r] ? 0 : tpos + 1;
  }
}

// Final Linear(H -> 1): one wave per row, fp64 accumulation, rounded once to f32.
__global__ __launch_bounds__(256) void k_value_head(int rows, const float* __restrict__ h, int ldh, int H,
                                                    const float* __restrict__ w, const float* __restrict__ b,
                                                    float* __restrict__ v) {
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* x = h + (long long)r * ldh;
  double s = 0.0;
  for (int k = lane; k < H; k += 64) s += (double)x[k] * (double)w[k];
  s = wave_sum(s);
  if (lane == 0) v[r] = (float)s + b[0];
}

// discount_sum + GAE / standard advantages (process_samples.py:3-45), one thread per lane,
// backward in time.  ret_run/adv_run restart at every trajectory end.
__global__ __launch_bounds__(256) void k_gae(Grid g, const uint8_t* __restrict__ end, const float* __restrict__ rew,
                                             const int64_t* __restrict__ rbase, long long rstride,
                                             const float* __restrict__ v, double gamma, double gl,
                                             double* __restrict__ ret, double* __restrict__ adv) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= g.L) return;
  const int n = g.length(l);
  const long long rb = rbase ? rbase[l] : (long long)l;
  const float gamma_f = (float)gamma;  // numpy casts the scalar to the float32 array's type
  double ret_run = 0.0, adv_run = 0.0;
  float b_next = 0.f;
  bool seg_f32 = false;
  for (int t = n - 1; t >= 0; --t) {
    const long long r = g.row(t, l);
    int e = end[r];
    if (t == n - 1 && e == 0) e = 2;  // cut by the buffer: not terminated
    const float b = v[r];
    if (e != 0) {                      // last row of a trajectory
      ret_run = 0.0;
      adv_run = 0.0;
      // b1 = np.append(b, 0.0 if terminated else b[-1]): float64 when terminated (the 0.0
      // becomes a float64 array), float32 otherwise -> the deltas' precision per trajectory
      seg_f32 = (e == 2);
      b_next = seg_f32 ? b : 0.f;
    }
    const float x = rew[rb + (long long)t * rstride];
    ret_run = (double)x + gamma * ret_run;  // run_sum = x[t] + gamma*run_sum (float64)
    ret[r] = ret_run;
    if (gl >= 0.0) {
      double delta;                         // rewards + gamma*b1[1:] - b1[:-1]
      if (seg_f32) {
        const float gb = gamma_f * b_next;
        const float s = x + gb;
        delta = (double)(s - b);
      } else {
        delta = ((double)x + gamma * (double)b_next) - (double)b;
      }
      adv_run = delta + gl * adv_run;       // discount_sum(td, gamma*lambda) in float64
      adv[r] = adv_run;
    } else {
      adv[r] = ret_run - (double)b;         // returns - baseline
    }
    b_next = b;
  }
}

// (adv - mean) / (std + eps) over the grid's rows (np.mean / np.std, population std), in two
// launches over the whole chip: the flat element range is cut into nb contiguous chunks of `ch`
// elements (a multiple of 1024; a fixed partition: deterministic), and
//   k_whiten_part: workgroup b reduces its chunk's count, sum and -- about its own mean, a second
//     pass over the chunk (L1/L2-resident) -- sum of squared deviations M2_b (fixed order: thread
//     strides, waves, then the 16 wave parts in order) into part[b];
//   k_whiten_apply: every workgroup combines the nb parts in block order (Chan et al.'s pairwise
//     update: mean = sum / n, M2 = sum_b M2_b + n_b (mean_b - mean)^2; the same bits in every
//     workgroup), std = sqrt(M2 / n), and writes its chunk; workgroup 0 writes stats.
// (Round 4's one-workgroup form: 25 us for 40 960 advantages, profiles/r05c_npg_timeline.txt.)
constexpr int WCH = 4096;  // elements per workgroup when the chunks fit AMX_WHITEN_MAXB workgroups

__device__ inline bool whiten_elem(const Grid& g, bool flat, long long i, long long end, long long& r) {
  if (i >= end) return false;
  if (flat) {
    r = i;
    return true;
  }
  const int t = (int)(i / g.L), l = (int)(i % g.L);
  if (t >= g.length(l)) return false;
  r = g.row(t, l);
  return true;
}

// fixed-order sum over the workgroup's 1024 threads (wave butterflies, then the 16 wave parts)
__device__ inline double block_sum(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < 16; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(1024) void k_whiten_part(Grid g, const double* __restrict__ adv, long long ch,
                                                      double* __restrict__ part) {
  __shared__ double red[16];
  const long long total = (long long)g.T * g.L;
  const bool flat = g.T == 1 && g.len == nullptr && g.base == nullptr;
  const long long c0 = (long long)blockIdx.x * ch, c1 = c0 + ch < total ? c0 + ch : total;
  double s = 0.0, cnt = 0.0;
  for (long long i = c0 + threadIdx.x; i < c1; i += 1024) {
    long long r = 0;
    if (whiten_elem(g, flat, i, c1, r)) {
      s += adv[r];
      cnt += 1.0;
    }
  }
  const double sum = block_sum(s, red);
  const double n = block_sum(cnt, red);
  const double m = n > 0.0 ? sum / n : 0.0;
  double q = 0.0;
  for (long long i = c0 + threadIdx.x; i < c1; i += 1024) {
    long long r = 0;
    if (whiten_elem(g, flat, i, c1, r)) {
      const double d = adv[r] - m;
      q += d * d;
    }
  }
  const double m2 = block_sum(q, red);
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = n;
    part[3 * blockIdx.x + 1] = sum;
    part[3 * blockIdx.x + 2] = m2;
  }
}

__global__ __launch_bounds__(1024) void k_whiten_apply(Grid g, const double* __restrict__ adv,
                                                       const double* __restrict__ part, int nb, long long ch,
                                                       double eps, double* __restrict__ out,
                                                       double* __restrict__ stats) {
  const long long total = (long long)g.T * g.L;
  const bool flat = g.T == 1 && g.len == nullptr && g.base == nullptr;
  double n = 0.0, sum = 0.0;
  for (int b = 0; b < nb; ++b) {  // every thread the same fixed order (broadcast loads)
    n += part[3 * b];
    sum += part[3 * b + 1];
  }
  const double mean = n > 0.0 ? sum / n : 0.0;
  double m2 = 0.0;
  for (int b = 0; b < nb; ++b) {
    const double nbk = part[3 * b];
    if (nbk > 0.0) {
      const double d = part[3 * b + 1] / nbk - mean;
      m2 += part[3 * b + 2] + nbk * d * d;
    }
  }
  const double sd = n > 0.0 ? sqrt(m2 / n) : 0.0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && stats) {
    stats[0] = mean;
    stats[1] = sd;
  }
  const double den = sd + eps;
  const long long c0 = (long long)blockIdx.x * ch, c1 = c0 + ch < total ? c0 + ch : total;
  for (long long i = c0 + threadIdx.x; i < c1; i += 1024) {
    long long r = 0;
    if (whiten_elem(g, flat, i, c1, r)) out[r] = (adv[r] - mean) / den;
  }
}

int check_grid(const char* fn, int T, int L, long long stride) {
  AMX_CHECK_ARG(T >= 0 && L >= 0, "%s: T=%d L=%d", fn, T, L);
  AMX_CHECK_ARG(stride >= 0, "%s: stride=%lld", fn, stride);
  return AMX_OK;
}

}  // namespace

extern "C" int amx_value_features(amx_ctx* ctx, int T, int L, const int32_t* len, const int32_t* t0,
                                  const int64_t* base, long long stride, const uint8_t* end, const double* obs,
                                  int ldo, float* feat, int ldf, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_value_features: null ctx");
  int rc = check_grid("amx_value_features", T, L, stride);
  if (rc) return rc;
  const int S = ctx->S, kf = amx::round_up(S + 4, AMX_K_TILE);
  AMX_CHECK_ARG(end && obs && feat, "amx_value_features: null pointer");
  AMX_CHECK_ARG(ldo >= S && ldf >= kf, "amx_value_features: ldo=%d (S=%d) ldf=%d (need >= %d)", ldo, S, ldf, kf);
  if (T == 0 || L == 0) return AMX_OK;
  Grid g{T, L, len, base, stride};
  hipLaunchKernelGGL(k_value_features, dim3((L + 3) / 4), dim3(256), 0, (hipStream_t)stream, g, t0, end, obs, ldo, S,
                     kf, feat, ldf);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_value_head(amx_ctx* ctx, int rows, const float* h, int ldh, int H, const float* w,
                              const float* b, float* v, void* stream) {
  AMX_CHECK_ARG(ctx && h && w && b && v, "amx_value_head: null pointer");
  AMX_CHECK_ARG(rows >= 0 && H > 0 && ldh >= H, "amx_value_head: rows=%d H=%d ldh=%d", rows, H, ldh);
  if (rows == 0) return AMX_OK;
  hipLaunchKernelGGL(k_value_head, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, rows, h, ldh, H, w, b, v);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_gae(amx_ctx* ctx, int T, int L, const int32_t* len, const int64_t* base, long long stride,
                       const uint8_t* end, const float* rew, const int64_t* rbase, long long rstride, const float* v,
                       double gamma, double gamma_lambda, double* ret, double* adv, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_gae: null ctx");
  int rc = check_grid("amx_gae", T, L, stride);
  if (rc) return rc;
  AMX_CHECK_ARG(end && rew && v && ret && adv, "amx_gae: null pointer");
  AMX_CHECK_ARG(rstride >= 0, "amx_gae: rstride=%lld", rstride);
  if (T == 0 || L == 0) return AMX_OK;
  Grid g{T, L, len, base, stride};
  hipLaunchKernelGGL(k_gae, dim3((L + 255) / 256), dim3(256), 0, (hipStream_t)stream, g, end, rew, rbase, rstride, v,
                     gamma, gamma_lambda, ret, adv);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_adv_whiten(amx_ctx* ctx, int T, int L, const int32_t* len, const int64_t* base,
                              long long stride, const double* adv, double eps, double* out, double* stats,
                              void* stream) {
  AMX_CHECK_ARG(ctx, "amx_adv_whiten: null ctx");
  int rc = check_grid("amx_adv_whiten", T, L, stride);
  if (rc) return rc;
  AMX_CHECK_ARG(adv && out, "amx_adv_whiten: null pointer");
  const long long total = (long long)T * L;
  long long ch = WCH;  // chunk per workgroup: WCH, or larger (multiples of 1024) beyond MAXB workgroups
  if ((total + ch - 1) / ch > AMX_WHITEN_MAXB) ch = ((total + AMX_WHITEN_MAXB - 1) / AMX_WHITEN_MAXB + 1023) / 1024 * 1024;
  const long long nb = total > 0 ? (total + ch - 1) / ch : 1;
  Grid g{T, L, len, base, stride};
  hipLaunchKernelGGL(k_whiten_part, dim3((int)nb), dim3(1024), 0, (hipStream_t)stream, g, adv, ch,
                     ctx->d_whiten_part);
  AMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_whiten_apply, dim3((int)nb), dim3(1024), 0, (hipStream_t)stream, g, adv, ctx->d_whiten_part,
                     (int)nb, ch, eps, out, stats);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
