// Context lifetime, configuration and error reporting of the amx C ABI.
#include <stdarg.h>
#include <stdlib.h>

#include "amx_common.h"

namespace amx {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace amx

extern "C" const char* amx_last_error(void) { return amx::g_err; }
extern "C" int amx_abi_version(void) { return AMX_ABI_VERSION; }

extern "C" amx_ctx* amx_create(int device, int S, int A, int n_models, int hidden, int n_hidden,
                               int feat_dim) {
  if (S <= 0 || A <= 0 || n_models <= 0 || n_models > AMX_MAX_MODELS || hidden <= 0 ||
      hidden % 128 != 0 || n_hidden < 0 || feat_dim <= 0 || feat_dim % 128 != 0) {
    amx::set_error("amx_create: bad dims S=%d A=%d M=%d H=%d L=%d F=%d (H, F must be multiples of 128, M <= %d)",
                   S, A, n_models, hidden, n_hidden, feat_dim, AMX_MAX_MODELS);
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    amx::set_error("amx_create: hipSetDevice(%d) failed", device);
    return nullptr;
  }
  amx_ctx* c = (amx_ctx*)calloc(1, sizeof(amx_ctx));
  if (!c) {
    amx::set_error("amx_create: out of host memory");
    return nullptr;
  }
  c->device = device;
  hipDeviceProp_t prop;
  c->n_cus = (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
                 ? prop.multiProcessorCount : 256;
  c->S = S;
  c->A = A;
  c->M = n_models;
  c->H = hidden;
  c->L = n_hidden;
  c->F = feat_dim;
  c->k0_pad = amx::round_up(S + A, AMX_K_TILE);
  c->ldk = c->k0_pad + n_hidden * hidden;
  c->n_out_pad = amx::round_up(S, AMX_ROW_TILE);
  c->k_rff_pad = amx::round_up(2 * S, AMX_K_TILE);
  if (hipMalloc((void**)&c->d_norm, sizeof(float) * (4 * S + 2 * A)) != hipSuccess) {
    free(c);
    amx::set_error("amx_create: hipMalloc of normalizers failed");
    return nullptr;
  }
  // amx_adv_whiten's per-block partials (allocated here: the launch stays graph-capturable)
  if (hipMalloc((void**)&c->d_whiten_part, sizeof(double) * 3 * AMX_WHITEN_MAXB) != hipSuccess) {
    (void)hipFree(c->d_norm);
    free(c);
    amx::set_error("amx_create: hipMalloc of the whitening partials failed");
    return nullptr;
  }
  return c;
}

extern "C" int amx_destroy(amx_ctx* c) {
  if (!c) return AMX_OK;
  if (c->d_norm) (void)hipFree(c->d_norm);
  if (c->d_motion) (void)hipFree(c->d_motion);
  if (c->d_npg_scratch) (void)hipFree(c->d_npg_scratch);
  if (c->d_whiten_part) (void)hipFree(c->d_whiten_part);
  free(c);
  return AMX_OK;
}

extern "C" int amx_layout(const amx_ctx* c, int* k0_pad, int* ldk, int* n_out_pad, int* k_rff_pad) {
  AMX_CHECK_ARG(c, "amx_layout: null ctx");
  if (k0_pad) *k0_pad = c->k0_pad;
  if (ldk) *ldk = c->ldk;
  if (n_out_pad) *n_out_pad = c->n_out_pad;
  if (k_rff_pad) *k_rff_pad = c->k_rff_pad;
  return AMX_OK;
}

extern "C" int amx_set_normalizers(amx_ctx* c, const float* mu_s, const float* sd_s, const float* mu_a,
                                   const float* sd_a, const float* mu_d, const float* sd_d) {
  AMX_CHECK_ARG(c && mu_s && sd_s && mu_a && sd_a && mu_d && sd_d, "amx_set_normalizers: null argument");
  const int S = c->S, A = c->A;
  float* h = (float*)malloc(sizeof(float) * (4 * S + 2 * A));
  AMX_CHECK_ARG(h, "amx_set_normalizers: out of host memory");
  // device layout: mu_s | sd_s | mu_a | sd_a | mu_d | sd_d
  memcpy(h, mu_s, sizeof(float) * S);
  memcpy(h + S, sd_s, sizeof(float) * S);
  memcpy(h + 2 * S, mu_a, sizeof(float) * A);
  memcpy(h + 2 * S + A, sd_a, sizeof(float) * A);
  memcpy(h + 2 * S + 2 * A, mu_d, sizeof(float) * S);
  memcpy(h + 3 * S + 2 * A, sd_d, sizeof(float) * S);
  hipError_t e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipMemcpy(c->d_norm, h, sizeof(float) * (4 * S + 2 * A), hipMemcpyHostToDevice);
  free(h);
  AMX_CHECK_HIP(e);
  c->have_norm = 1;
  return AMX_OK;
}

extern "C" int amx_set_termination(amx_ctx* c, int n_bodies, const int32_t* body_id, const int32_t* shape,
                                   const double* p0, const double* p1, int record_all_world,
                                   int record_world_root_pos, int pos_dim, int rot_dim, int horizon,
                                   int vel_check, int vel_offset, double vel_thresh, int record_vel_as_pos,
                                   double sampling_rate) {
  AMX_CHECK_ARG(c, "amx_set_termination: null ctx");
  AMX_CHECK_ARG(n_bodies >= 0 && n_bodies <= AMX_MAX_BODIES, "amx_set_termination: n_bodies=%d out of range",
                n_bodies);
  AMX_CHECK_ARG(n_bodies == 0 || (body_id && shape && p0 && p1), "amx_set_termination: null body table");
  AMX_CHECK_ARG(!vel_check || (vel_offset >= 0 && vel_offset <= c->S), "amx_set_termination: vel_offset");
  AMX_CHECK_ARG(!(vel_check && record_vel_as_pos) || sampling_rate != 0.0,
                "amx_set_termination: sampling_rate must be nonzero");
  amx_termination t;
  memset(&t, 0, sizeof(t));
  t.n = n_bodies;
  for (int i = 0; i < n_bodies; ++i) {
    // sim_env.py:103-104: offset = (pos_dim + rot_dim) * body + 1 (ob[0] is the root y)
    const int off = (pos_dim + rot_dim) * body_id[i] + 1;
    AMX_CHECK_ARG(shape[i] >= 0 && shape[i] <= 2, "amx_set_termination: shape[%d]=%d", i, shape[i]);
    AMX_CHECK_ARG(off + pos_dim + 1 < c->S || shape[i] == AMX_SHAPE_BOX,
                  "amx_set_termination: body %d indexes past the state (S=%d)", body_id[i], c->S);
    t.shape[i] = shape[i];
    t.y_index[i] = off + 1;                  // sim_env.py:182,185
    t.ny_index[i] = off + pos_dim + 1;       // sim_env.py:213
    // sim_env.py:181,223: the list index (not the body id) selects the root rule
    t.list_index_world[i] = (record_all_world || (i == 0 && record_world_root_pos)) ? 1 : 0;
    const double radius = 0.5 * p0[i];      // sim_env.py:188,199
    t.thresh[i] = radius + 0.0001;          // sim_env.py:189,236
    t.half_h[i] = 0.5 * p1[i];              // 0.5 * cylinder_height (then * norm_y), :215
    t.neg_half_h[i] = -0.5 * p1[i];         // -0.5 * cylinder_height (then * norm_y), :216
  }
  t.horizon = horizon;
  t.vel_check = vel_check;
  t.vel_offset = vel_offset;
  t.vel_thresh = vel_thresh;
  t.record_vel_as_pos = record_vel_as_pos;
  t.sampling_rate = sampling_rate;
  c->term = t;
  c->have_term = 1;
  return AMX_OK;
}
