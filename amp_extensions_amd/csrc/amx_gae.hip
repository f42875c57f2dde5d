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

// (adv - mean) / (std + eps) over the grid's rows: one 1024-thread block, fixed order
// (thread-strided partial sums, then an LDS tree), two passes as np.mean / np.std.
__global__ __launch_bounds__(1024) void k_adv_whiten(Grid g, const double* __restrict__ adv, double eps,
                                                     double* __restrict__ out, double* __restrict__ stats) {
  __shared__ double red[1024];
  __shared__ double s_mean, s_std;
  const long long total = (long long)g.T * g.L;
  // a flat vector (one row of L, no lengths / bases: DeviceNPG's whitening): element i is row i
  // and every element counts -- the same thread-strided order without the 64-bit index division
  const bool flat = g.T == 1 && g.len == nullptr && g.base == nullptr;
  double s = 0.0, cnt = 0.0;
  if (flat) {
#pragma unroll 8
    for (long long i = threadIdx.x; i < total; i += 1024) {
      s += adv[i];
      cnt += 1.0;
    }
  } else {
    for (long long i = threadIdx.x; i < total; i += 1024) {
      const int t = (int)(i / g.L), l = (int)(i % g.L);
      if (t < g.length(l)) {
        s += adv[g.row(t, l)];
        cnt += 1.0;
      }
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double sum = red[0];
  __syncthreads();
  red[threadIdx.x] = cnt;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double n = red[0];
  if (threadIdx.x == 0) s_mean = n > 0.0 ? sum / n : 0.0;
  __syncthreads();
  const double mean = s_mean;
  double q = 0.0;
  if (flat) {
#pragma unroll 8
    for (long long i = threadIdx.x; i < total; i += 1024) {
      const double d = adv[i] - mean;
      q += d * d;
    }
  } else {
    for (long long i = threadIdx.x; i < total; i += 1024) {
      const int t = (int)(i / g.L), l = (int)(i % g.L);
      if (t < g.length(l)) {
        const double d = adv[g.row(t, l)] - mean;
        q += d * d;
      }
    }
  }
  __syncthreads();
  red[threadIdx.x] = q;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    s_std = n > 0.0 ? sqrt(red[0] / n) : 0.0;
    if (stats) {
      stats[0] = mean;
      stats[1] = s_std;
    }
  }
  __syncthreads();
  const double den = s_std + eps;
  if (flat) {
#pragma unroll 8
    for (long long i = threadIdx.x; i < total; i += 1024) out[i] = (adv[i] - mean) / den;
  } else {
    for (long long i = threadIdx.x; i < total; i += 1024) {
      const int t = (int)(i / g.L), l = (int)(i % g.L);
      if (t < g.length(l)) {
        const long long r = g.row(t, l);
        out[r] = (adv[r] - mean) / den;
      }
    }
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
  Grid g{T, L, len, base, stride};
  hipLaunchKernelGGL(k_adv_whiten, dim3(1), dim3(1024), 0, (hipStream_t)stream, g, adv, eps, out, stats);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
