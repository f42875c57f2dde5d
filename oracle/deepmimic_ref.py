"""CPU restatement of SimEnv.reset's DeepMimicCore path (TEST INFRASTRUCTURE ONLY).

SimEnv.reset (gym-simenv/gym_simenv/envs/sim_env.py:270-285) asks DeepMimicCore for the
state of the simulated character reset to time t of the reference motion.  The C++ core is
not buildable here (Bullet 2.88, Eigen 3.3.7, GL are absent), so this module restates, in
float64 numpy, the code that path runs (paths relative to
deepmimic/deepmimic/DeepMimicCore/):

  Motion::Load / PostProcessFrames / BuildFrameVel / CalcFrame / CalcFrameVel /
      CalcIndexBlend (anim/Motion.cpp:104-135, 167-305, 415-530)
  KinTree::LerpPoses / CalcVel / PostProcessPose / JointWorldTrans / ChildParentTrans* /
      BuildOriginTrans / CalcHeading (anim/KinTree.cpp:1082-1135, 1518-1720, 1806-1880)
  KinCharacter::CalcPose (StandardizeQuat of the root, anim/KinCharacter.cpp:573-596)
  SceneImitate::ResetKinCharTime + SyncCharacters (scenes/SceneImitate.cpp:469-533) with
      SimEnv's default reset_args (no noise, radian 0: AddNoise is a no-op)
  SceneSimChar::ResetSceneTime -> SetCharRandPlacement (plane ground: root x, z -> 0,
      scenes/SceneSimChar.cpp:545-562, sim/Ground.cpp:154-159) -> ResolveCharGroundIntersect
      (scenes/SceneSimChar.cpp:565-607, 0.001 pad) over the body shapes' AABBs
  CtController::BuildStatePose / BuildStateVel (sim/CtController.cpp:378-495) with the
      humanoid3d_rot_ctrl flags (RecordWorldRootPos false, RecordWorldRootRot true)
  cMathUtil quaternion helpers (util/MathUtil.cpp:141-640)

Third-party algorithms restated from their published sources (absent here):
  * Eigen 3.3.7 QuaternionBase::slerp (Eigen/src/Geometry/Quaternion.h) and the
    quaternion-vector product (v + w*uv + u x uv, uv = 2 u x v);
  * Bullet 2.88 getAabb of btSphereShape (center +- radius), btCapsuleShape (Y-up half
    extents (r, r + h/2, r) through |R|) and btBoxShape (half extents through |R|; the box's
    margin is folded into its implicit dimensions, so the AABB is the geometric one).
Body velocities are the kinematic world velocities of the body attach points
(KinTree::CalcBodyPartVel / RBDUtil::CalcWorldVel, sim/RBDUtil.cpp:225-495): the simulated
character is set to the kinematic pose and velocity at reset.  Parity is UNPINNED against
the reference: no reference output of this path exists without the C++ core.
"""
from __future__ import annotations

import json
import math

import numpy as np

JOINT_TYPES = {"revolute": 0, "planar": 1, "prismatic": 2, "fixed": 3, "spherical": 4, "none": 5}
PARAM_SIZE = {0: 1, 1: 3, 2: 1, 3: 0, 4: 4, 5: 7}
SHAPES = {"box": 0, "capsule": 1, "sphere": 2, "cylinder": 3, "plane": 4}


def load_character(src):
    """src: a character file path, its JSON text, or the parsed dict."""
    d = src if isinstance(src, dict) else (json.loads(src) if src.lstrip().startswith("{") else json.load(open(src)))
    joints = []
    off = 0
    for j in d["Skeleton"]["Joints"]:
        t = JOINT_TYPES[j["Type"]] if j["Parent"] != -1 else JOINT_TYPES["none"]
        size = PARAM_SIZE[t]
        attach = np.array([j["AttachX"], j["AttachY"], j["AttachZ"]], float)
        if j["Parent"] == -1:
            attach[:] = 0.0  # KinTree::PostProcessJointMat zeroes the root attach point
        joints.append(dict(type=t, parent=int(j["Parent"]), offset=off, size=size, attach=attach,
                           theta=np.array([j["AttachThetaX"], j["AttachThetaY"], j["AttachThetaZ"]], float)))
        off += size
    bodies = []
    for b in d["BodyDefs"]:
        bodies.append(dict(shape=SHAPES[b["Shape"]], attach=np.array([b["AttachX"], b["AttachY"], b["AttachZ"]], float),
                           theta=np.array([b["AttachThetaX"], b["AttachThetaY"], b["AttachThetaZ"]], float),
                           param=np.array([b["Param0"], b["Param1"], b["Param2"]], float)))
    return joints, bodies, off


# ---- quaternion helpers (w, x, y, z), cMathUtil / Eigen -----------------------------------
def qmul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz, aw * bz + az * bw + ax * by - ay * bx])


def qconj(q):
    return np.array([q[0], -q[1], -q[2], -q[3]])


def qrot(q, v):
    """Eigen Quaternion * Vector3: uv = 2 (u x v); v + w uv + u x uv."""
    u = q[1:]
    uv = np.cross(u, v)
    uv = uv + uv
    return v + q[0] * uv + np.cross(u, uv)


def slerp(q0, q1, t):
    """Eigen 3.3.7 QuaternionBase::slerp."""
    one = 1.0 - np.finfo(float).eps
    d = float(np.dot(q0, q1))
    absd = abs(d)
    if absd >= one:
        s0, s1 = 1.0 - t, t
    else:
        th = math.acos(absd)
        st = math.sin(th)
        s0 = math.sin((1.0 - t) * th) / st
        s1 = math.sin(t * th) / st
    if d < 0:
        s1 = -s1
    return s0 * q0 + s1 * q1


def rotmat(q):
    """cMathUtil::RotateMat(quaternion), 3x3."""
    w, x, y, z = q
    sqw, sqx, sqy, sqz = w * w, x * x, y * y, z * z
    invs = 1 / (sqx + sqy + sqz + sqw)
    m = np.zeros((3, 3))
    m[0, 0] = (sqx - sqy - sqz + sqw) * invs
    m[1, 1] = (-sqx + sqy - sqz + sqw) * invs
    m[2, 2] = (-sqx - sqy + sqz + sqw) * invs
    t1, t2 = x * y, z * w
    m[1, 0] = 2.0 * (t1 + t2) * invs
    m[0, 1] = 2.0 * (t1 - t2) * invs
    t1, t2 = x * z, y * w
    m[2, 0] = 2.0 * (t1 - t2) * invs
    m[0, 2] = 2.0 * (t1 + t2) * invs
    t1, t2 = y * z, x * w
    m[2, 1] = 2.0 * (t1 + t2) * invs
    m[1, 2] = 2.0 * (t1 - t2) * invs
    return m


def rotmat_axis(axis, theta):
    c, s = math.cos(theta), math.sin(theta)
    x, y, z = axis
    return np.array([[c + x * x * (1 - c), x * y * (1 - c) - z * s, x * z * (1 - c) + y * s],
                     [y * x * (1 - c) + z * s, c + y * y * (1 - c), y * z * (1 - c) - x * s],
                     [z * x * (1 - c) - y * s, z * y * (1 - c) + x * s, c + z * z * (1 - c)]])


def mat_to_quat(m):
    """cMathUtil::RotMatToQuaternion."""
    tr = m[0, 0] + m[1, 1] + m[2, 2]
    if tr > 0:
        S = math.sqrt(tr + 1.0) * 2
        return np.array([0.25 * S, (m[2, 1] - m[1, 2]) / S, (m[0, 2] - m[2, 0]) / S, (m[1, 0] - m[0, 1]) / S])
    if m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
        S = math.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
        return np.array([(m[2, 1] - m[1, 2]) / S, 0.25 * S, (m[0, 1] + m[1, 0]) / S, (m[0, 2] + m[2, 0]) / S])
    if m[1, 1] > m[2, 2]:
        S = math.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
        return np.array([(m[0, 2] - m[2, 0]) / S, (m[0, 1] + m[1, 0]) / S, 0.25 * S, (m[1, 2] + m[2, 1]) / S])
    S = math.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
    return np.array([(m[1, 0] - m[0, 1]) / S, (m[0, 2] + m[2, 0]) / S, (m[1, 2] + m[2, 1]) / S, 0.25 * S])


def quat_to_axis_angle(q):
    """cMathUtil::QuaternionToAxisAngle."""
    q1 = q
    if q1[0] > 1:
        q1 = q1 / np.linalg.norm(q1)
    sin_t = math.sqrt(1 - q1[0] * q1[0])
    if sin_t > 0.000001:
        th = 2 * math.acos(q1[0])
        th = normalize_angle(th)
        return q1[1:] / sin_t, th
    return np.array([0.0, 0.0, 1.0]), 0.0


def normalize_angle(th):
    """cMathUtil::NormalizeAngle: wrap into (-pi, pi]."""
    th = math.fmod(th, 2 * math.pi)
    if th < -math.pi:
        th += 2 * math.pi
    elif th > math.pi:
        th -= 2 * math.pi
    return th


def quat_vel(q0, q1, dt):
    """CalcQuaternionVel: world-frame angular velocity of q0 -> q1 (q_diff = q1 q0*)."""
    axis, th = quat_to_axis_angle(qmul(q1, qconj(q0)))
    return (th / dt) * axis


def quat_vel_rel(q0, q1, dt):
    """CalcQuaternionVelRel: angular velocity in the frame of q0 (q_diff = q0* q1)."""
    axis, th = quat_to_axis_angle(qmul(qconj(q0), q1))
    return (th / dt) * axis


# ---- motion ------------------------------------------------------------------------------
class Motion:
    def __init__(self, src, joints):
        """src: a motion file path or the parsed {"Loop", "Frames"} dict."""
        d = src if isinstance(src, dict) else json.load(open(src))
        self.loop = d.get("Loop", "none") != "none"
        raw = np.array(d["Frames"], float)
        self.joints = joints
        durs = raw[:, 0].copy()
        frames = raw[:, 1:].copy()
        t, times = 0.0, np.zeros(len(raw))
        off = frames[0, 0:3].copy()
        off[1] = 0.0
        for f in range(len(raw)):   # PostProcessFrames (Motion.cpp:415-442)
            times[f] = t
            t += durs[f]
            frames[f, 0:3] -= off
            self._post_process(frames[f])
        self.times, self.frames = times, frames
        n = len(frames)
        vels = np.zeros_like(frames)   # BuildFrameVel (Motion.cpp:167-188)
        for f in range(n - 1):
            vels[f] = self.calc_vel(frames[f], frames[f + 1], times[f + 1] - times[f])
        if n > 1:
            vels[n - 1] = vels[n - 2]
        self.vels = vels
        self.duration = times[-1]
        self.cycle_delta = frames[-1, 0:3] - frames[0, 0:3]
        self.cycle_delta[1] = 0.0

    def _post_process(self, pose):
        pose[3:7] /= np.linalg.norm(pose[3:7])
        for j in self.joints[1:]:
            if j["type"] == 4:
                o = j["offset"]
                pose[o:o + 4] /= np.linalg.norm(pose[o:o + 4])

    def calc_vel(self, p0, p1, dt):
        """KinTree::CalcVel (KinTree.cpp:1518-1556)."""
        out = np.zeros_like(p0)
        out[0:3] = (p1[0:3] - p0[0:3]) / dt
        out[3:6] = quat_vel(p0[3:7], p1[3:7], dt)
        out[6] = 0.0
        for j in self.joints[1:]:
            o, s = j["offset"], j["size"]
            if j["type"] == 4:
                out[o:o + 3] = quat_vel_rel(p0[o:o + 4], p1[o:o + 4], dt)
                out[o + 3] = 0.0
            elif s > 0:
                out[o:o + s] = (p1[o:o + s] - p0[o:o + s]) / dt
        return out

    def index_blend(self, time):
        """Motion::CalcIndexBlend (Motion.cpp:495-522)."""
        if not self.loop:
            if time <= 0:
                return 0, 0.0
            if time >= self.duration:
                return len(self.frames) - 2, 1.0
        count = int(math.floor(time / self.duration))
        if not self.loop:
            count = min(max(count, 0), 1)
        time -= count * self.duration
        idx = int(np.searchsorted(self.times, time, side="right")) - 1
        t0, t1 = self.times[idx], self.times[idx + 1]
        return idx, (time - t0) / (t1 - t0)

    def pose(self, time):
        """MotionController::CalcPose + KinCharacter::CalcPose (origin identity)."""
        idx, blend = self.index_blend(time)
        blend = min(max(blend, 0.0), 1.0)   # Motion::BlendFrames saturates
        p0, p1 = self.frames[idx], self.frames[idx + 1]
        out = np.zeros_like(p0)
        out[0:3] = (1 - blend) * p0[0:3] + blend * p1[0:3]
        q = slerp(p0[3:7], p1[3:7], blend)
        out[3:7] = q / np.linalg.norm(q)
        for j in self.joints[1:]:
            o, s = j["offset"], j["size"]
            if j["type"] == 4:
                out[o:o + 4] = slerp(p0[o:o + 4], p1[o:o + 4], blend)
            elif s > 0:
                out[o:o + s] = (1 - blend) * p0[o:o + s] + blend * p1[o:o + s]
        if self.loop:
            out[0:3] += math.floor(time / self.duration) * self.cycle_delta
        if out[3] < 0:   # StandardizeQuat
            out[3:7] = -out[3:7]
        return out

    def vel(self, time):
        if not self.loop and time >= self.duration:
            return np.zeros(self.frames.shape[1])
        idx, blend = self.index_blend(time)
        return (1.0 - blend) * self.vels[idx] + blend * self.vels[idx + 1]


# ---- kinematics, reset, state ------------------------------------------------------------
def forward_kinematics(joints, pose, vel):
    """Joint world rotations R_j, origins o_j, angular velocities w_j and origin velocities
    v_j (JointWorldTrans / RBDUtil::CalcWorldVel)."""
    J = len(joints)
    R, o, w, v = [None] * J, [None] * J, [None] * J, [None] * J
    for j, jt in enumerate(joints):
        if jt["parent"] < 0:
            R[j] = rotmat(pose[3:7])
            o[j] = pose[0:3].copy()
            w[j] = vel[3:6].copy()
            v[j] = vel[0:3].copy()
            continue
        p = jt["parent"]
        o[j] = o[p] + R[p] @ jt["attach"]
        off = jt["offset"]
        if jt["type"] == 4:
            R[j] = R[p] @ rotmat(pose[off:off + 4])
            w[j] = w[p] + R[j] @ vel[off:off + 3]
        elif jt["type"] == 0:
            R[j] = R[p] @ rotmat_axis((0.0, 0.0, 1.0), pose[off])
            w[j] = w[p] + R[j] @ np.array([0.0, 0.0, vel[off]])
        else:   # fixed
            R[j] = R[p].copy()
            w[j] = w[p].copy()
        v[j] = v[p] + np.cross(w[p], o[j] - o[p])
    return R, o, w, v


def body_aabb_min_y(body, R, c):
    """Bullet 2.88 getAabb (min y) of the body's collision shape at rotation R, center c."""
    sh, prm = body["shape"], body["param"]
    if sh == 2:   # sphere: diameter Param0
        return c[1] - 0.5 * prm[0]
    if sh == 1:   # capsule: diameter Param0, cylinder height Param1, Y-up
        half = np.array([0.5 * prm[0], 0.5 * prm[0] + 0.5 * prm[1], 0.5 * prm[0]])
    else:         # box
        half = 0.5 * prm
    return c[1] - np.abs(R[1]) @ half


# ---- reset noise: cKinCharacter::AddNoise (anim/KinCharacter.cpp:340-470) ------------------
NOISE_ROT_SLOTS = 48   # uniforms reserved per reset for RandomRotatePoseVel's draws
HIPS_ANKLES = (3, 5, 9, 11)   # humanoid3d joints RandomRotatePoseVel never perturbs
KNEES = (4, 10)


def euler_to_quat(x, y, z):
    """cMathUtil::EulerToQuaternion = AxisAngleToQuaternion(EulerToAxisAngle(euler))
    (util/MathUtil.cpp:347-381, 423-466)."""
    xs, xc, ys, yc, zs, zc = math.sin(x), math.cos(x), math.sin(y), math.cos(y), math.sin(z), math.cos(z)
    c = (yc * zc + xs * ys * zs + xc * zc + xc * yc - 1) * 0.5
    c = min(max(c, -1.0), 1.0)
    th = math.acos(c)
    if abs(th) < 0.00001:
        axis = np.array([0.0, 0.0, 1.0])
    else:
        m21 = xs * yc - xc * ys * zs + xs * zc
        m02 = xc * ys * zc + xs * zs + ys
        m10 = yc * zs - xs * ys * zc + xc * zs
        den = math.sqrt(m21 * m21 + m02 * m02 + m10 * m10)
        axis = np.array([m21 / den, m02 / den, m10 / den])
    ch, sh = math.cos(th / 2), math.sin(th / 2)
    return np.array([ch, sh * axis[0], sh * axis[1], sh * axis[2]])


def add_noise(joints, pose, vel, ra, u_rot, u_pv):
    """cKinCharacter::AddNoise(noise_bef_rot, min, max, radian, rot_vel_w_pose, vel_noise, interp,
    knee_rot) on the kinematic pose / velocity at the reset time (SceneImitate::ResetKinCharTime,
    scenes/SceneImitate.cpp:469-489), with its uniforms injected: u_rot feeds RandomRotatePoseVel's
    cMathUtil::RandDouble(-radian, radian) draws (gRand's mRandGen) in call order, u_pv
    AddNoisePoseVel's RandDoubleEigen(size, min, max) draws (gRand's mGen): pose elements, then
    velocity elements.  A draw u in [0, 1) gives lo + u (hi - lo) (cRand::RandDouble,
    util/Rand.cpp:35-46; std::uniform_real_distribution).  Quaternions are (w, x, y, z) pose
    segments (cMathUtil::VecToQuat / QuatToVec); velocity segments are rotated as the reference
    does, the 4-vector (w_x, w_y, w_z, pad) read as a quaternion (w = w_x).  The joint indices of
    the knee / hip / ankle exclusions are humanoid3d's, as hard-coded in the reference, and so is
    the velocity-noise revolute test `!(j == 4 || j != 10) || knee_rot` (only joint 10 unless
    knee_rot).  Returns new (pose, vel)."""
    pose, vel = np.array(pose, float), np.array(vel, float)
    lo, hi, r = float(ra["noise_min"]), float(ra["noise_max"]), float(ra["radian"])
    it_r, it_p = iter(u_rot), iter(u_pv)

    def rnd():
        return -r + next(it_r) * (r - (-r))

    def pose_vel():   # AddNoisePoseVel (KinCharacter.cpp:354-366)
        if lo == 0 and hi == 0:
            return
        n = len(pose)
        pose[:] = pose + np.array([lo + next(it_p) * (hi - lo) for _ in range(n)])
        vel[:] = vel + np.array([lo + next(it_p) * (hi - lo) for _ in range(n)])

    def rotate():   # RandomRotatePoseVel (KinCharacter.cpp:367-470)
        if r == 0:
            return
        a = rnd()
        qy = np.array([math.cos(a / 2), 0.0, math.sin(a / 2), 0.0])   # AxisAngleToQuaternion((0,1,0), a)
        # cCharacter::RotateRoot (anim/Character.cpp:210-216): new = normalize(rot * root_rot),
        # then the virtual cKinCharacter::SetRootRotation (KinCharacter.cpp:259-264):
        # dq = new * root_rot^-1 and RotateOrigin(dq) (KinCharacter.cpp:300-337), which sets the
        # root rotation to normalize(dq * root_rot) and rotates the root's linear velocity and
        # angular velocity by dq (QuatRotVec: xyz rotated, the 4th slot of gRotDim written 0)
        old = pose[3:7].copy()
        new = qmul(qy, old)
        new = new / np.linalg.norm(new)
        dq = qmul(new, qconj(old))
        q = qmul(dq, old)
        pose[3:7] = q / np.linalg.norm(q)
        vel[0:3] = qrot(dq, vel[0:3])
        vel[3:6] = qrot(dq, vel[3:6])
        vel[6] = 0.0
        interp = float(ra["interp"])
        vel[0:3] = interp * vel[0:3]   # GetRootVel / SetRootVel (gPosDim)
        vel[3:7] = interp * vel[3:7]   # GetRootAngVel / SetRootAngVel (gRotDim = 4)
        for jt in joints[1:]:
            o, sz = jt["offset"], jt["size"]
            vel[o:o + sz] = interp * vel[o:o + sz]
        for j in range(1, len(joints)):
            o, t = joints[j]["offset"], joints[j]["type"]
            if t == 0:
                if j not in KNEES or ra["knee_rot"]:
                    pose[o] = pose[o] + rnd()
            elif t == 4 and j not in HIPS_ANKLES:
                ps, th, ph = rnd(), rnd(), rnd()
                qr = euler_to_quat(ps, th, ph)
                pose[o:o + 4] = qmul(qr, pose[o:o + 4])
                if ra["rot_vel_w_pose"]:
                    vel[o:o + 4] = qmul(qr, vel[o:o + 4])
        if ra["vel_noise"]:
            ps, th, ph = rnd(), rnd(), rnd()
            vel[3:7] = qmul(euler_to_quat(ps, th, ph), vel[3:7])
            for j in range(1, len(joints)):
                o, t = joints[j]["offset"], joints[j]["type"]
                if t == 0:
                    if not (j == 4 or j != 10) or ra["knee_rot"]:
                        vel[o] = vel[o] + rnd()
                elif t == 4 and j not in HIPS_ANKLES:
                    ps, th, ph = rnd(), rnd(), rnd()
                    vel[o:o + 4] = qmul(euler_to_quat(ps, th, ph), vel[o:o + 4])
        pose[3:7] = pose[3:7] / np.linalg.norm(pose[3:7])   # KinTree::PostProcessPose
        for jt in joints[1:]:
            if jt["type"] == 4:
                o = jt["offset"]
                pose[o:o + 4] = pose[o:o + 4] / np.linalg.norm(pose[o:o + 4])

    if ra["noise_bef_rot"]:
        pose_vel()
        rotate()
    else:
        rotate()
        pose_vel()
    return pose, vel


def noise_draws(joints, ra):
    """(uniforms RandomRotatePoseVel consumes, uniforms AddNoisePoseVel consumes) for reset_args ra."""
    nr = 0
    if float(ra["radian"]) != 0:
        nr = 1
        for j in range(1, len(joints)):
            t = joints[j]["type"]
            if t == 0:
                nr += int(j not in KNEES or bool(ra["knee_rot"]))
            elif t == 4 and j not in HIPS_ANKLES:
                nr += 3
        if ra["vel_noise"]:
            nr += 3
            for j in range(1, len(joints)):
                t = joints[j]["type"]
                if t == 0:
                    nr += int((not (j == 4 or j != 10)) or bool(ra["knee_rot"]))
                elif t == 4 and j not in HIPS_ANKLES:
                    nr += 3
    D = sum(j["size"] for j in joints)
    npv = 0 if float(ra["noise_min"]) == 0 and float(ra["noise_max"]) == 0 else 2 * D
    return nr, npv


def reset_state(joints, bodies, motion, time, record_world_root_pos=False, record_world_root_rot=True,
                record_all_world=False, ground_pad=0.001, resolve=True, noise=None, u_rot=(), u_pv=()):
    """The 226-d state SimEnv.reset records after reset_time(time); `resolve` = reset_args'
    'resolve' (SceneSimChar::ResetSceneTime, scenes/SceneSimChar.cpp:714-716); `noise` = the
    reset_args of AddNoise with its injected uniforms u_rot / u_pv (add_noise), applied to the
    kinematic pose / velocity before the placement and the ground resolve
    (SceneSimChar.cpp:699-716: ResetCharactersTime, then InitCharacterPos, then resolve)."""
    pose = motion.pose(time)
    vel = motion.vel(time)
    if noise is not None:
        pose, vel = add_noise(joints, pose, vel, noise, u_rot, u_pv)
    pose[0] = 0.0   # SetCharRandPlacement on the plane: root x, z -> 0 (y kept)
    pose[2] = 0.0
    R, o, w, v = forward_kinematics(joints, pose, vel)
    bpos = [o[j] + R[j] @ bodies[j]["attach"] for j in range(len(joints))]
    # ResolveCharGroundIntersect
    min_viol = 0.0
    for j in range(len(joints) if resolve else 0):
        min_viol = min(min_viol, body_aabb_min_y(bodies[j], R[j], bpos[j]) - ground_pad)
    if min_viol < 0:
        pose[1] += -min_viol
        for j in range(len(joints)):
            o[j][1] += -min_viol
            bpos[j][1] += -min_viol
    # CtController::BuildStatePose
    root_pos = pose[0:3]
    rd = qrot(pose[3:7], np.array([1.0, 0.0, 0.0]))
    heading = math.atan2(-rd[2], rd[0])
    Rh = rotmat_axis((0.0, 1.0, 0.0), -heading)
    origin = np.array([root_pos[0], 0.0, root_pos[2]])
    qh = mat_to_quat(Rh)

    def to_origin(x):
        return Rh @ (x - origin)

    root_rel = to_origin(root_pos)
    n = len(joints)
    S = 1 + n * 9 + n * 6
    out = np.zeros(S)
    out[0] = root_rel[1]
    for i in range(n):
        p = bpos[i].copy()
        if not record_all_world and (not record_world_root_pos or i != 0):
            p = to_origin(p) - root_rel
        out[9 * i + 1:9 * i + 4] = p
        q = mat_to_quat(R[i])
        if not record_all_world and (not record_world_root_rot or i != 0):
            q = qmul(qh, q)
        out[9 * i + 4:9 * i + 7] = qrot(q, np.array([0.0, 1.0, 0.0]))
        out[9 * i + 7:9 * i + 10] = qrot(q, np.array([1.0, 0.0, 0.0]))
    # CtController::BuildStateVel
    base = 1 + n * 9
    for i in range(n):
        lv = v[i] + np.cross(w[i], bpos[i] - o[i])
        av = w[i]
        if not record_all_world and (not record_world_root_rot or i != 0):
            lv, av = Rh @ lv, Rh @ av
        out[base + 6 * i:base + 6 * i + 3] = lv
        out[base + 6 * i + 3:base + 6 * i + 6] = av
    return out


# ---- AMP observation features (scenes/SceneImitateAMP.cpp:287-475) -----------------------
def end_effectors(char_src):
    d = char_src if isinstance(char_src, dict) else json.loads(char_src)
    return [j["ID"] for j in d["Skeleton"]["Joints"] if j.get("IsEndEffector", 0)]


def motion_frame(M, time):
    """Motion::CalcFrame (raw clip blend: no cycle offset, no root StandardizeQuat)."""
    idx, blend = M.index_blend(time)
    blend = min(max(blend, 0.0), 1.0)
    p0, p1 = M.frames[idx], M.frames[idx + 1]
    out = (1 - blend) * p0 + blend * p1
    q = slerp(p0[3:7], p1[3:7], blend)
    out[3:7] = q / np.linalg.norm(q)
    for j in M.joints[1:]:
        if j["type"] == 4:
            o = j["offset"]
            out[o:o + 4] = slerp(p0[o:o + 4], p1[o:o + 4], blend)
    return out


def heading_rot(q):
    """KinTree::CalcHeadingRot: rotation about y by -heading (3x3)."""
    rd = qrot(q, np.array([1.0, 0.0, 0.0]))
    return rotmat_axis((0.0, 1.0, 0.0), -math.atan2(-rd[2], rd[0]))


def amp_obs_pose(joints, bodies, ee, pose, Rh, local_root=False, ground_h=0.0):
    """RecordAMPObsPose (SceneImitateAMP.cpp:370-439)."""
    out = [pose[1] - ground_h]
    R0 = rotmat(pose[3:7])
    if local_root:
        R0 = Rh @ R0
    out += list(R0[:, 1]) + list(R0[:, 0])   # tan-norm: R e_y (norm), R e_x (tan)
    for j in joints[1:]:
        o = j["offset"]
        if j["type"] == 4:
            L = rotmat(pose[o:o + 4])
            out += list(L[:, 1]) + list(L[:, 0])
        elif j["size"] > 0:
            out += list(pose[o:o + j["size"]])
    R, org, _, _ = forward_kinematics(joints, pose, np.zeros(len(pose)))
    for e in ee:
        p = org[e] + R[e] @ bodies[e]["attach"] - pose[0:3]
        out += list(Rh @ p)
    return np.array(out)


def amp_obs_vel(joints, vel, Rh, local_root=False):
    """RecordAMPObsVel (SceneImitateAMP.cpp:441-475)."""
    v, w = vel[0:3], vel[3:6]
    if local_root:
        v, w = Rh @ v, Rh @ w
    return np.concatenate([v, w, vel[7:]])


def amp_obs(joints, bodies, ee, prev_pose, prev_vel, pose, vel, local_root=False, ground_h=0.0):
    """BuildAMPObs (SceneImitateAMP.cpp:352-368): [pose, prev pose, vel, prev vel] in the
    current pose's heading frame."""
    Rh = heading_rot(pose[3:7])
    return np.concatenate([amp_obs_pose(joints, bodies, ee, pose, Rh, local_root, ground_h),
                           amp_obs_pose(joints, bodies, ee, prev_pose, Rh, local_root, ground_h),
                           amp_obs_vel(joints, vel, Rh, local_root), amp_obs_vel(joints, prev_vel, Rh, local_root)])


def expert_amp_obs(joints, bodies, ee, M, time, dt=1.0 / 30, local_root=False):
    """RecordAMPObsExpert (SceneImitateAMP.cpp:167-193) at a given clip time."""
    return amp_obs(joints, bodies, ee, motion_frame(M, time - dt), M.vel(time - dt), motion_frame(M, time),
                   M.vel(time), local_root)


def reset_pose_vel(joints, bodies, M, time, ground_pad=0.001):
    """(pose, vel) of the simulated character after reset_time(time): the pose reset_state
    records (placement on the plane and the ground lift applied)."""
    pose = M.pose(time)
    vel = M.vel(time)
    pose[0] = pose[2] = 0.0
    R, o, w, v = forward_kinematics(joints, pose, vel)
    lows = [body_aabb_min_y(bodies[j], R[j], o[j] + R[j] @ bodies[j]["attach"]) - ground_pad
            for j in range(len(joints))]
    lift = -min(0.0, min(lows))
    pose[1] += lift
    return pose, vel


# ---- AMP features from two recorded SimEnv states ----------------------------------------
# The learned-dynamics SimEnv records CtController states (no joint quaternions), so the
# AMP observation of a transition (s, s') is built from what the state holds: rotations from
# the tangent-normal pairs (R = [tan, nrm, tan x nrm]), joint velocity parameters from the
# body angular velocities, end-effector offsets from the body positions.  On a state that
# reset_state recorded these equal the quantities amp_obs reads from (pose, vel); this is the
# restatement of amx_motion.hip's kin_from_state / amp_pose_part / amp_vel_part used to check
# the device on arbitrary (dynamics-predicted) states.
def _tn_mat(nt):
    nrm, tan = np.asarray(nt[0:3], float), np.asarray(nt[3:6], float)
    return np.column_stack([tan, nrm, np.cross(tan, nrm)])


def state_kin(joints, ee, s):
    n = len(joints)
    base = 1 + 9 * n
    Rw0 = _tn_mat(s[4:10])
    Rh = rotmat_axis((0.0, 1.0, 0.0), -math.atan2(-Rw0[2, 0], Rw0[0, 0]))
    R = [Rh @ Rw0] + [_tn_mat(s[9 * i + 4:9 * i + 10]) for i in range(1, n)]
    w0 = np.asarray(s[base + 3:base + 6], float)
    w = [Rh @ w0] + [np.asarray(s[base + 6 * i + 3:base + 6 * i + 6], float) for i in range(1, n)]
    v0 = np.asarray(s[base:base + 3], float) - np.cross(w0, Rh.T @ np.asarray(s[1:4], float))
    jv = []
    for i in range(1, n):
        j = joints[i]
        if j["type"] in (0, 4):
            wl = R[i].T @ (w[i] - w[j["parent"]])
            jv += [wl[0], wl[1], wl[2], 0.0] if j["type"] == 4 else [wl[2]]
    return dict(root_y=s[0], Rw0=Rw0, Rh=Rh, R=R, v0=v0, w0=w0, jv=np.array(jv),
                ee=[np.asarray(s[9 * e + 1:9 * e + 4], float) for e in ee])


def state_amp_obs(joints, ee, s_prev, s_cur, local_root=False):
    kp, kc = state_kin(joints, ee, s_prev), state_kin(joints, ee, s_cur)
    Rc = kc["Rh"]

    def pose_part(k):
        R0 = Rc @ k["Rw0"] if local_root else k["Rw0"]
        out = [k["root_y"]] + list(R0[:, 1]) + list(R0[:, 0])
        for i in range(1, len(joints)):
            j = joints[i]
            if j["type"] in (0, 4):
                L = k["R"][j["parent"]].T @ k["R"][i]
                out += list(L[:, 1]) + list(L[:, 0]) if j["type"] == 4 else [math.atan2(L[1, 0], L[0, 0])]
        Rx = Rc @ k["Rh"].T
        for e in k["ee"]:
            out += list(Rx @ e)
        return np.array(out)

    def vel_part(k):
        v, w = k["v0"], k["w0"]
        if local_root:
            v, w = Rc @ v, Rc @ w
        return np.concatenate([v, w, k["jv"]])

    return np.concatenate([pose_part(kc), pose_part(kp), vel_part(kc), vel_part(kp)])
