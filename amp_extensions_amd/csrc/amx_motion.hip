// SimEnv.reset from the reference motion, on the device: the state the
// simulated humanoid records after DeepMimicCore's reset_time(t) (gym-simenv/gym_simenv/envs/
// sim_env.py:270-285 -> DeepMimicCore.cpp:85-88), computed per lane from the motion clip:
//
//   pose(t), vel(t)   Motion::CalcFrame / CalcFrameVel (anim/Motion.cpp:267-305): frame
//                     index + blend (CalcIndexBlend :495-522), KinTree::LerpPoses
//                     (anim/KinTree.cpp:1577-1620: root slerp + normalize, spherical slerp,
//                     revolute lerp; Eigen 3.3.7's slerp), root StandardizeQuat
//                     (KinCharacter::CalcPose, anim/KinCharacter.cpp:573-596), loop cycle
//                     offset (MotionController::CalcPose); frame velocities lerped
//   placement         SetCharRandPlacement on the plane ground: root x, z -> 0
//                     (scenes/SceneSimChar.cpp:545-562, sim/Ground.cpp:154-159)
//   kinematics        JointWorldTrans (KinTree.cpp:1126-1135 + ChildParentTrans*), body attach
//                     points, world body velocities (RBDUtil::CalcWorldVel)
//   ground resolve    ResolveCharGroundIntersect (scenes/SceneSimChar.cpp:565-607): lift the
//                     root by the deepest AABB violation (0.001 pad) of the body shapes
//                     (Bullet 2.88 getAabb of sphere / capsule / box)
//   state             CtController::BuildStatePose / BuildStateVel (sim/CtController.cpp:
//                     378-495): root y, heading-frame body positions, tangent-normal body
//                     rotations, heading-frame velocities (world for the root when
//                     RecordWorldRootRot)
//
// The clip is preprocessed once on the host (amp_extensions_amd/motion.py: PostProcessFrames
// and BuildFrameVel, Motion.cpp:167-188, 415-442) and uploaded as one fp64 blob
// (amx_set_motion).  One thread per lane, fp64 throughout; the per-joint frames live in the
// thread's private memory (resets are rare after the first: a few lanes per step).
#include "amx_common.h"

namespace {

constexpr int MAXJ = 16;   // joints / bodies
constexpr int MAXD = 96;   // pose / velocity dofs
constexpr int HDR = 16;
enum { JT_REVOLUTE = 0, JT_FIXED = 3, JT_SPHERICAL = 4, JT_ROOT = 5 };
enum { SH_BOX = 0, SH_CAPSULE = 1, SH_SPHERE = 2 };

struct MView {  // views into the device blob
  const double* h;
  const double* joints;  // [J][8]: type, parent, offset, size, ax, ay, az, -
  const double* bodies;  // [J][8]: shape, ax, ay, az, p0, p1, p2, valid
  const double* times;   // [F]
  const double* frames;  // [F][D]
  const double* vels;    // [F][D]
  int J, D, F;
  __device__ MView(const double* b) {
    h = b;
    J = (int)h[0];
    D = (int)h[1];
    F = (int)h[2];
    joints = b + HDR;
    bodies = joints + 8 * J;
    times = bodies + 8 * J;
    frames = times + F;
    vels = frames + (long long)F * D;
  }
};

struct Q { double w, x, y, z; };
struct V3 { double x, y, z; };

__device__ inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ inline V3 scale(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
// 3x3 row-major
__device__ inline V3 mv(const double* m, V3 v) {
  return {m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
          m[6] * v.x + m[7] * v.y + m[8] * v.z};
}
__device__ inline void mm(const double* a, const double* b, double* o) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) o[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
// cMathUtil::RotateMat(quaternion) (util/MathUtil.cpp:212-251)
__device__ inline void qmat(Q q, double* m) {
  const double sqw = q.w * q.w, sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z;
  const double invs = 1 / (sqx + sqy + sqz + sqw);
  m[0] = (sqx - sqy - sqz + sqw) * invs;
  m[4] = (-sqx + sqy - sqz + sqw) * invs;
  m[8] = (-sqx - sqy + sqz + sqw) * invs;
  double t1 = q.x * q.y, t2 = q.z * q.w;
  m[3] = 2.0 * (t1 + t2) * invs;
  m[1] = 2.0 * (t1 - t2) * invs;
  t1 = q.x * q.z; t2 = q.y * q.w;
  m[6] = 2.0 * (t1 - t2) * invs;
  m[2] = 2.0 * (t1 + t2) * invs;
  t1 = q.y * q.z; t2 = q.x * q.w;
  m[7] = 2.0 * (t1 + t2) * invs;
  m[5] = 2.0 * (t1 - t2) * invs;
}
// cMathUtil::RotateMat(axis, theta) for the unit axes used here
__device__ inline void axis_mat(V3 a, double th, double* m) {
  const double c = cos(th), s = sin(th), x = a.x, y = a.y, z = a.z;
  m[0] = c + x * x * (1 - c); m[1] = x * y * (1 - c) - z * s; m[2] = x * z * (1 - c) + y * s;
  m[3] = y * x * (1 - c) + z * s; m[4] = c + y * y * (1 - c); m[5] = y * z * (1 - c) - x * s;
  m[6] = z * x * (1 - c) - y * s; m[7] = z * y * (1 - c) + x * s; m[8] = c + z * z * (1 - c);
}
// cMathUtil::RotMatToQuaternion (util/MathUtil.cpp:310-345)
__device__ inline Q mat_q(const double* m) {
  const double tr = m[0] + m[4] + m[8];
  if (tr > 0) {
    const double S = sqrt(tr + 1.0) * 2;
    return {0.25 * S, (m[7] - m[5]) / S, (m[2] - m[6]) / S, (m[3] - m[1]) / S};
  }
  if (m[0] > m[4] && m[0] > m[8]) {
    const double S = sqrt(1.0 + m[0] - m[4] - m[8]) * 2;
    return {(m[7] - m[5]) / S, 0.25 * S, (m[1] + m[3]) / S, (m[2] + m[6]) / S};
  }
  if (m[4] > m[8]) {
    const double S = sqrt(1.0 + m[4] - m[0] - m[8]) * 2;
    return {(m[2] - m[6]) / S, (m[1] + m[3]) / S, 0.25 * S, (m[5] + m[7]) / S};
  }
  const double S = sqrt(1.0 + m[8] - m[0] - m[4]) * 2;
  return {(m[3] - m[1]) / S, (m[2] + m[6]) / S, (m[5] + m[7]) / S, 0.25 * S};
}
__device__ inline Q qmul(Q a, Q b) {
  return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
          a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
// Eigen: q * v = v + w*uv + u x uv, uv = 2 (u x v)
__device__ inline V3 qrot(Q q, V3 v) {
  const V3 u = {q.x, q.y, q.z};
  V3 uv = cross(u, v);
  uv = add(uv, uv);
  return add(add(v, scale(uv, q.w)), cross(u, uv));
}
// Eigen 3.3.7 QuaternionBase::slerp
__device__ inline Q slerp(Q a, Q b, double t) {
  const double one = 1.0 - 2.220446049250313e-16;
  const double d = a.w * b.w + a.x * b.x + a.y * b.y + a.z * b.z;
  const double ad = fabs(d);
  double s0, s1;
  if (ad >= one) {
    s0 = 1.0 - t;
    s1 = t;
  } else {
    const double th = acos(ad), st = sin(th);
    s0 = sin((1.0 - t) * th) / st;
    s1 = sin(t * th) / st;
  }
  if (d < 0) s1 = -s1;
  return {s0 * a.w + s1 * b.w, s0 * a.x + s1 * b.x, s0 * a.y + s1 * b.y, s0 * a.z + s1 * b.z};
}
__device__ inline Q qnorm(Q q) {
  const double n = sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  return {q.w / n, q.x / n, q.y / n, q.z / n};
}
__device__ inline Q ldq(const double* p) { return {p[0], p[1], p[2], p[3]}; }

// The recorded state at motion time `time` (see the file comment).  out: [S] = 1 + 15 J.
__device__ void motion_state(const MView& m, double time, int flags, double* __restrict__ out) {
  const double dur = m.h[4];
  const bool loop = m.h[3] != 0.0;
  // ---- Motion::CalcIndexBlend ---------------------------------------------------------------
  int idx;
  double blend;
  double cycles = 0.0;
  if (!loop && time <= 0.0) {
    idx = 0; blend = 0.0;
  } else if (!loop && time >= dur) {
    idx = m.F - 2; blend = 1.0;
  } else {
    double cnt = floor(time / dur);
    if (!loop) cnt = fmin(fmax(cnt, 0.0), 1.0);
    cycles = cnt;
    const double tt = time - cnt * dur;
    int lo = 0, hi = m.F;  // upper_bound
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (m.times[mid] <= tt) lo = mid + 1; else hi = mid;
    }
    idx = lo - 1;
    if (idx > m.F - 2) idx = m.F - 2;
    if (idx < 0) idx = 0;
    blend = (tt - m.times[idx]) / (m.times[idx + 1] - m.times[idx]);
  }
  const double lerp = fmin(fmax(blend, 0.0), 1.0);  // BlendFrames saturates
  const double* f0 = m.frames + (long long)idx * m.D;
  const double* f1 = f0 + m.D;
  const double* v0 = m.vels + (long long)idx * m.D;
  const double* v1 = v0 + m.D;
  double pose[MAXD], vel[MAXD];
  for (int i = 0; i < m.D; ++i) {
    pose[i] = (1 - lerp) * f0[i] + lerp * f1[i];
    vel[i] = (!loop && time >= dur) ? 0.0 : (1.0 - blend) * v0[i] + blend * v1[i];
  }
  {
    Q q = qnorm(slerp(ldq(f0 + 3), ldq(f1 + 3), lerp));
    if (q.w < 0) q = {-q.w, -q.x, -q.y, -q.z};  // StandardizeQuat
    pose[3] = q.w; pose[4] = q.x; pose[5] = q.y; pose[6] = q.z;
  }
  for (int j = 1; j < m.J; ++j) {
    const double* jt = m.joints + 8 * j;
    if ((int)jt[0] == JT_SPHERICAL) {
      const int o = (int)jt[2];
      const Q q = slerp(ldq(f0 + o), ldq(f1 + o), lerp);
      pose[o] = q.w; pose[o + 1] = q.x; pose[o + 2] = q.y; pose[o + 3] = q.z;
    }
  }
  if (loop) {
    pose[0] += cycles * m.h[8];
    pose[1] += cycles * m.h[9];
    pose[2] += cycles * m.h[10];
  }
  pose[0] = 0.0;  // random placement on the plane: root x, z = 0
  pose[2] = 0.0;
  // ---- kinematics ---------------------------------------------------------------------------
  double R[MAXJ][9];
  V3 o[MAXJ], w[MAXJ], v[MAXJ], bp[MAXJ];
  for (int j = 0; j < m.J; ++j) {
    const double* jt = m.joints + 8 * j;
    const int type = (int)jt[0], par = (int)jt[1], off = (int)jt[2];
    if (par < 0) {
      qmat(ldq(pose + 3), R[j]);
      o[j] = {pose[0], pose[1], pose[2]};
      w[j] = {vel[3], vel[4], vel[5]};
      v[j] = {vel[0], vel[1], vel[2]};
    } else {
      o[j] = add(o[par], mv(R[par], {jt[4], jt[5], jt[6]}));
      double L[9];
      if (type == JT_SPHERICAL) {
        qmat(ldq(pose + off), L);
        mm(R[par], L, R[j]);
        w[j] = add(w[par], mv(R[j], {vel[off], vel[off + 1], vel[off + 2]}));
      } else if (type == JT_REVOLUTE) {
        axis_mat({0.0, 0.0, 1.0}, pose[off], L);
        mm(R[par], L, R[j]);
        w[j] = add(w[par], mv(R[j], {0.0, 0.0, vel[off]}));
      } else {  // fixed
        for (int k = 0; k < 9; ++k) R[j][k] = R[par][k];
        w[j] = w[par];
      }
      v[j] = add(v[par], cross(w[par], sub(o[j], o[par])));
    }
    const double* bd = m.bodies + 8 * j;
    bp[j] = add(o[j], mv(R[j], {bd[1], bd[2], bd[3]}));
  }
  // ---- ResolveCharGroundIntersect -------------------------------------------------------------
  double min_viol = 0.0;
  const double pad = m.h[11];
  for (int j = 0; j < m.J; ++j) {
    const double* bd = m.bodies + 8 * j;
    if (bd[7] == 0.0) continue;
    const int sh = (int)bd[0];
    double ext;
    if (sh == SH_SPHERE) {
      ext = 0.5 * bd[4];
    } else {
      const double hx = 0.5 * bd[4], hy = sh == SH_CAPSULE ? 0.5 * bd[4] + 0.5 * bd[5] : 0.5 * bd[5];
      const double hz = sh == SH_CAPSULE ? 0.5 * bd[4] : 0.5 * bd[6];
      ext = fabs(R[j][3]) * hx + fabs(R[j][4]) * hy + fabs(R[j][5]) * hz;
    }
    min_viol = fmin(min_viol, bp[j].y - ext - pad);
  }
  if (min_viol < 0) {
    pose[1] += -min_viol;
    for (int j = 0; j < m.J; ++j) {
      o[j].y += -min_viol;
      bp[j].y += -min_viol;
    }
  }
  // ---- CtController::BuildStatePose / BuildStateVel ---------------------------------------------
  const bool world_root_pos = flags & 1, world_root_rot = flags & 2, all_world = flags & 4;
  const V3 rd = qrot(ldq(pose + 3), {1.0, 0.0, 0.0});
  const double heading = atan2(-rd.z, rd.x);
  double Rh[9];
  axis_mat({0.0, 1.0, 0.0}, -heading, Rh);
  const Q qh = mat_q(Rh);
  const V3 origin = {pose[0], 0.0, pose[2]};
  const V3 root_rel = mv(Rh, sub({pose[0], pose[1], pose[2]}, origin));
  out[0] = root_rel.y;
  const int n = m.J;
  for (int i = 0; i < n; ++i) {
    V3 p = bp[i];
    if (!all_world && (!world_root_pos || i != 0)) p = sub(mv(Rh, sub(p, origin)), root_rel);
    out[9 * i + 1] = p.x; out[9 * i + 2] = p.y; out[9 * i + 3] = p.z;
    Q q = mat_q(R[i]);
    if (!all_world && (!world_root_rot || i != 0)) q = qmul(qh, q);
    const V3 nrm = qrot(q, {0.0, 1.0, 0.0}), tan = qrot(q, {1.0, 0.0, 0.0});
    out[9 * i + 4] = nrm.x; out[9 * i + 5] = nrm.y; out[9 * i + 6] = nrm.z;
    out[9 * i + 7] = tan.x; out[9 * i + 8] = tan.y; out[9 * i + 9] = tan.z;
  }
  const int base = 1 + 9 * n;
  for (int i = 0; i < n; ++i) {
    V3 lv = add(v[i], cross(w[i], sub(bp[i], o[i])));
    V3 av = w[i];
    if (!all_world && (!world_root_rot || i != 0)) {
      lv = mv(Rh, lv);
      av = mv(Rh, av);
    }
    double* d = out + base + 6 * i;
    d[0] = lv.x; d[1] = lv.y; d[2] = lv.z; d[3] = av.x; d[4] = av.y; d[5] = av.z;
  }
}

__global__ __launch_bounds__(64) void k_motion_states(const double* __restrict__ blob, const double* __restrict__ times,
                                                      int B, int flags, double* __restrict__ ob, long long ldo) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const MView m(blob);
  motion_state(m, times[b], flags, ob + (long long)b * ldo);
}

// SimEnv.reset on masked lanes with motion states: reset_count/model_idx/num_steps as in
// k_reset (sim_env.py:277, 282-283); t = times[b] or uniform(0, duration) from
// Philox(seed, lane, reset#) (np_random.uniform(low=0, high=time_max), :276).
__global__ __launch_bounds__(64) void k_reset_motion(const double* __restrict__ blob, const uint8_t* __restrict__ mask,
                                                     const double* __restrict__ times, uint32_t k0, uint32_t k1,
                                                     int flags, const double* ob_src, double* ob_out,
                                                     int32_t* num_steps, int32_t* model_idx, int32_t* reset_count,
                                                     double* t_out, int S, int M, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const bool do_reset = (mask == nullptr) || mask[b] != 0;
  if (!do_reset) {
    if (ob_src != ob_out)
      for (int j = 0; j < S; ++j) ob_out[(long long)b * S + j] = ob_src[(long long)b * S + j];
    if (t_out) t_out[b] = -1.0;
    return;
  }
  const MView m(blob);
  const int rc = reset_count[b] + 1;
  double t;
  if (times) {
    t = times[b];
  } else {
    const amx::u32x4 r = amx::philox4x32_10({(uint32_t)b, (uint32_t)rc, 0u, amx::kTagMotion}, k0, k1);
    t = 0.0 + (m.h[4] - 0.0) * amx::u53(r.x, r.y);
  }
  motion_state(m, t, flags, ob_out + (long long)b * S);
  reset_count[b] = rc;
  model_idx[b] = rc % M;
  num_steps[b] = 0;
  if (t_out) t_out[b] = t;
}

}  // namespace

extern "C" int amx_set_motion(amx_ctx* c, const double* blob, long long n) {
  AMX_CHECK_ARG(c && blob && n > HDR, "amx_set_motion: null ctx/blob or n=%lld", n);
  const int J = (int)blob[0], D = (int)blob[1], F = (int)blob[2];
  AMX_CHECK_ARG(J > 0 && J <= MAXJ && D > 7 && D <= MAXD && F >= 2, "amx_set_motion: J=%d (<= %d) D=%d (<= %d) F=%d",
                J, MAXJ, D, MAXD, F);
  AMX_CHECK_ARG(n == HDR + 16LL * J + F + 2LL * F * D, "amx_set_motion: blob has %lld doubles, expected %lld", n,
                HDR + 16LL * J + F + 2LL * F * D);
  AMX_CHECK_ARG(c->S == 1 + 15 * J, "amx_set_motion: state size S=%d != 1 + 15*J (%d)", c->S, 1 + 15 * J);
  AMX_CHECK_ARG(blob[4] > 0.0, "amx_set_motion: duration %g", blob[4]);
  for (int j = 0; j < J; ++j) {
    const double* jt = blob + HDR + 8 * j;
    const int type = (int)jt[0], par = (int)jt[1], off = (int)jt[2];
    AMX_CHECK_ARG((j == 0) == (par < 0) && par < j, "amx_set_motion: joint %d parent %d (joints must be ordered)", j,
                  par);
    AMX_CHECK_ARG(type == JT_REVOLUTE || type == JT_FIXED || type == JT_SPHERICAL || (j == 0 && type == JT_ROOT),
                  "amx_set_motion: joint %d type %d unsupported", j, type);
    AMX_CHECK_ARG(off >= 0 && off + (int)jt[3] <= D, "amx_set_motion: joint %d params past the frame", j);
  }
  AMX_CHECK_HIP(hipSetDevice(c->device));
  if (c->d_motion && c->motion_n != n) {
    AMX_CHECK_HIP(hipFree(c->d_motion));
    c->d_motion = nullptr;
  }
  if (!c->d_motion) {
    if (hipMalloc((void**)&c->d_motion, sizeof(double) * n) != hipSuccess) {
      amx::set_error("amx_set_motion: hipMalloc failed");
      return AMX_E_NOMEM;
    }
  }
  AMX_CHECK_HIP(hipMemcpy(c->d_motion, blob, sizeof(double) * n, hipMemcpyHostToDevice));
  c->motion_n = n;
  c->motion_J = J;
  c->motion_D = D;
  c->motion_F = F;
  c->motion_duration = blob[4];
  return AMX_OK;
}

extern "C" double amx_motion_duration(const amx_ctx* c) { return (c && c->d_motion) ? c->motion_duration : -1.0; }

extern "C" int amx_motion_states(amx_ctx* c, const double* times, int B, int flags, double* ob, long long ldo,
                                 void* stream) {
  AMX_CHECK_ARG(c && c->d_motion, "amx_motion_states: no motion set (amx_set_motion)");
  AMX_CHECK_ARG(times && ob && B >= 0 && ldo >= c->S, "amx_motion_states: bad arguments");
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_motion_states, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, c->d_motion, times, B,
                     flags, ob, ldo);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_reset_lanes_motion(amx_ctx* c, const uint8_t* mask, const double* times, uint64_t seed,
                                      int flags, const double* ob_src, double* ob_out, int32_t* num_steps,
                                      int32_t* model_idx, int32_t* reset_count, double* t_out, int B, void* stream) {
  AMX_CHECK_ARG(c && c->d_motion, "amx_reset_lanes_motion: no motion set (amx_set_motion)");
  AMX_CHECK_ARG(ob_out && num_steps && model_idx && reset_count && B >= 0, "amx_reset_lanes_motion: null pointer");
  AMX_CHECK_ARG(mask == nullptr || ob_src != nullptr, "amx_reset_lanes_motion: masked reset needs ob_src");
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_reset_motion, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, c->d_motion, mask, times,
                     (uint32_t)seed, (uint32_t)(seed >> 32), flags, ob_src, ob_out, num_steps, model_idx,
                     reset_count, t_out, c->S, c->M, B);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
