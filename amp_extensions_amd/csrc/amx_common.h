// Shared internals of libamx_hip: context, error plumbing, Philox RNG.
// Written for gfx950 (CDNA4, wave64).  Everything here is device-agnostic C++ plus
// HIP device helpers; the kernels live in amx_*.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/amx_hip.h"

struct amx_termination {
  int n;                                   // bodies checked
  int list_index_world[AMX_MAX_BODIES];    // 1 -> body y is recorded in world frame
  int y_index[AMX_MAX_BODIES];             // ob index of the body's y position
  int ny_index[AMX_MAX_BODIES];            // ob index of the capsule normal's y
  int shape[AMX_MAX_BODIES];
  double thresh[AMX_MAX_BODIES];           // 0.5*P0 + 0.0001, evaluated in host double
  double half_h[AMX_MAX_BODIES];           // 0.5*P1
  double neg_half_h[AMX_MAX_BODIES];       // -0.5*P1
  int horizon;
  int vel_check;
  int vel_offset;
  double vel_thresh;
  int record_vel_as_pos;
  double sampling_rate;
};

struct amx_ctx {
  int device;
  int n_cus;               // compute units of the device (tile selection: workgroups resident at once)
  int S, A, M, H, L, F;
  int k0_pad, ldk, n_out_pad, k_rff_pad;
  // device copies of the normalizers: mu_s, sd_s (S), mu_a, sd_a (A), mu_d, sd_d (S)
  float* d_norm;
  int have_norm;
  amx_termination term;
  int have_term;
  // reference motion for the motion-reset path (amx_set_motion): device copy of the blob
  double* d_motion;
  long long motion_n;
  int motion_J, motion_D, motion_F;
  double motion_duration;
  int amp_obs_size;          // AMP observation features per transition (0: no character)
  uint64_t* gemm_timer;      // amx_set_gemm_timer: [start, arrivals, ticks, forwards] or null
  float* split_scratch;      // amx_set_split_workspace: split-K partial tiles of the output layer
  long long split_floats;
  uint32_t* split_cnt;       //   and its per-tile arrival counters (zero when idle)
  int split_ncnt;
  int step_act_w8;           // amx_set_step_act_occupancy: k_step_act at two workgroups per CU (A/B)
  double* d_npg_scratch;     // amx_npg_reduce's run sums
  size_t npg_scratch_bytes;
  double* d_whiten_part;     // amx_adv_whiten's per-block (count, sum, M2): AMX_WHITEN_MAXB x 3
};

constexpr int AMX_WHITEN_MAXB = 1024;  // amx_adv_whiten: most workgroups of its first pass

namespace amx {

void set_error(const char* fmt, ...);

#define AMX_CHECK_ARG(cond, ...)              \
  do {                                        \
    if (!(cond)) {                            \
      ::amx::set_error(__VA_ARGS__);          \
      return AMX_E_INVAL;                     \
    }                                         \
  } while (0)

#define AMX_CHECK_HIP(expr)                                                         \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ::amx::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),       \
                       __FILE__, __LINE__);                                         \
      return AMX_E_HIP;                                                             \
    }                                                                               \
  } while (0)

#define AMX_CHECK_LAUNCH() AMX_CHECK_HIP(hipGetLastError())

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
static inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ---- Philox4x32-10 (Salmon et al., SC'11), key = 2x32, counter = 4x32 ------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(M0, c.x, hi0, lo0);
    mulhilo32(M1, c.z, hi1, lo1);
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// 53-bit uniform in [0, 1) from two 32-bit words (same construction as numpy's
// random_standard_uniform on MT19937 output: (a>>5, b>>6)).
__host__ __device__ inline double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// Stream tags in the 4th counter word keep the RNG streams of different kernels apart.
constexpr uint32_t kTagReset = 0x52534554u;   // 'RSET'
constexpr uint32_t kTagPolicy = 0x504F4C49u;  // 'POLI'
constexpr uint32_t kTagMotion = 0x4D4F5449u;  // 'MOTI'

}  // namespace amx
