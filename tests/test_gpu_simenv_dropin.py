"""SimEnv built the way run.py builds it (run.py:113-120: `gym.make('simenv-v0',
deepmimic_args=args.deepmimic, dynamic_ensemble=..., reset_args=...)`), with no extra keyword:
the reset source comes from the DeepMimic arg file's --character_files / --motion_file /
--char_ctrl_files (run_amp_humanoid3d_spinkick_args.txt:17,23-24), reset_args is honoured
(custom_time / time_max window, sim_env.py:76-77, 276; resolve, SceneSimChar.cpp:714-716).

The oracle is SimEnvRef (sim_env.py:140-285 restated) with its resets taken from
deepmimic_ref.reset_state, the CPU restatement of DeepMimicCore's reset_time(t) + record_state
(parity of that restatement against the C++ core is unpinned: DESIGN.md §5.1).  Reset draws
come from the reference's gym 0.26 np_random stream; per-step parity as test_gpu_configs'
configs[0] test: both sides step from the oracle's state, next states within 2e-5 of
max(1, |ref|), done flags exact, reset states within 1e-10."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import deepmimic_ref as DR
from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
S, A = 226, 28

# run.py:113-117 with milo/milo/arguments.py's defaults (custom_time False, time_min/max 0,
# resolve = not no_resolve, noise 0, radian 0, interp 1)
RUN_PY_RESET_ARGS = dict(custom_time=False, time_min=0, time_max=0, resolve=True, noise_bef_rot=False,
                         noise_min=0, noise_max=0, radian=0, rot_vel_w_pose=False, vel_noise=False, interp=1.0,
                         knee_rot=False)


def write_deepmimic_tree(root):
    """The arg file and the data files it names, laid out as the deepmimic package root
    (args/..., data/characters, data/motions, data/controllers), from the package's humanoid3d +
    spinkick bundle.  The arg file keeps the reference's structure (comment lines, first
    occurrence of a key wins)."""
    from amp_extensions_amd.motion import ReferenceMotion
    z = np.load(ReferenceMotion.DEFAULT_BUNDLE, allow_pickle=False)
    for d in ("args", "data/characters", "data/motions", "data/controllers"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    with open(os.path.join(root, "data/characters/humanoid3d.txt"), "w") as f:
        f.write(str(z["character_json"]))
    with open(os.path.join(root, "data/motions/humanoid3d_spinkick.txt"), "w") as f:
        json.dump({"Loop": str(z["loop"]), "Frames": z["frames"].tolist()}, f)
    with open(os.path.join(root, "data/controllers/humanoid3d_rot_ctrl.txt"), "w") as f:
        json.dump({"UpdateRate": 30, "EnablePhaseInput": False, "RecordWorldRootPos": False,
                   "RecordWorldRootRot": True}, f)
    args = os.path.join(root, "args/run_amp_humanoid3d_spinkick_args.txt")
    with open(args, "w") as f:
        f.write("--scene imitate_amp\n\n--num_update_substeps 10\n#Time lims here even in testing\n"
                "--time_lim_min 0.5\n--char_types general\n--character_files data/characters/humanoid3d.txt\n"
                "--fall_contact_bodies 0 1 2 3 4 6 7 8 9 10 12 13 14\n--char_ctrls ct_pd\n"
                "--char_ctrl_files data/controllers/humanoid3d_rot_ctrl.txt\n--kin_ctrl motion\n"
                "--motion_file data/motions/humanoid3d_spinkick.txt\n--motion_file data/motions/absent.txt\n"
                "#--model_files data/policies/none.ckpt\n")
    return args


@pytest.fixture(scope="module")
def setup(tmp_path_factory):
    import amp_extensions_amd as amx
    from amp_extensions_amd import synthetic as syn
    root = str(tmp_path_factory.mktemp("deepmimic"))
    args = write_deepmimic_tree(root)
    s, a, s2 = syn.offline(8000, S, A, 0)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ens_w = R.init_ensemble_weights(S, A, [512] * 4, 4, 100)
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=DEV)
    ens = amx.DeviceEnsemble(ctx, ens_w, norms)
    J, bodies, _ = DR.load_character(json.load(open(os.path.join(root, "data/characters/humanoid3d.txt"))))
    M = DR.Motion(json.load(open(os.path.join(root, "data/motions/humanoid3d_spinkick.txt"))), J)
    return amx, ens, ens_w, norms, args, J, bodies, M


def _rel(x, ref):
    return float((np.abs(x - ref) / np.maximum(1.0, np.abs(ref))).max())


def test_simenv_from_run_py_arguments_matches_oracle_trace(setup):
    """SimEnv(dynamic_ensemble=, deepmimic_args=, reset_args=run.py's) over 600 steps with
    resets: every reset state vs reset_state(t) at the reference's drawn t, every step vs
    SimEnvRef."""
    amx, ens, ens_w, norms, args, J, bodies, M = setup
    env = amx.SimEnv(dynamic_ensemble=ens, deepmimic_args=args, reset_args=RUN_PY_RESET_ARGS, seed=11)
    assert env.motion is not None and env.time_max == pytest.approx(M.duration)
    ref = R.SimEnvRef(ens_w, norms, horizon=300)
    rng = R.gym_np_random(11)  # env.seed_env(11)
    acts = np.random.RandomState(12).randn(600, A) * np.exp(-0.25)
    resets = 0

    def both_reset():
        o = env.reset()
        t = rng.uniform(low=0, high=M.duration)
        assert env.last_reset_time == t
        ref.reset(DR.reset_state(J, bodies, M, t))
        assert _rel(o, ref.ob) <= 1e-10
        ref.ob = o.copy()  # continue both from the same state
        return 1

    resets += both_reset()
    worst = 0.0
    for t in range(600):
        env.set_observation(ref.ob.copy())
        no, r, d, info = env.step(acts[t].copy())
        rno, _, rd, _ = ref.step(acts[t].copy())
        assert r == 0 and info == {}
        worst = max(worst, _rel(no, rno))
        assert d == rd, t
        if d:
            resets += both_reset()
    assert worst <= 2e-5, worst
    assert resets >= 3


def test_simenv_custom_time_window_and_no_resolve(setup):
    """reset_args custom_time / time_max: t ~ U(0, time_max) (time_min ignored by reset, as
    sim_env.py:276 ignores it); resolve False: no ground lift.  Reset states vs the oracle."""
    amx, ens, ens_w, norms, args, J, bodies, M = setup
    ra = dict(RUN_PY_RESET_ARGS, custom_time=True, time_min=0.2, time_max=0.4)
    env = amx.SimEnv(ens, deepmimic_args=args, reset_args=ra, seed=5)
    assert env.time_max == 0.4 and env.time_min == 0.2
    rng = R.gym_np_random(5)
    for _ in range(12):
        o = env.reset()
        t = rng.uniform(low=0, high=0.4)
        assert env.last_reset_time == t and t < 0.4
        assert _rel(o, DR.reset_state(J, bodies, M, t)) <= 1e-10
    env2 = amx.SimEnv(ens, deepmimic_args=args, reset_args=dict(RUN_PY_RESET_ARGS, resolve=False), seed=6)
    rng = R.gym_np_random(6)
    lifted = 0
    for _ in range(12):
        o = env2.reset()
        t = rng.uniform(low=0, high=M.duration)
        want = DR.reset_state(J, bodies, M, t, resolve=False)
        assert _rel(o, want) <= 1e-10
        lifted += not np.array_equal(want, DR.reset_state(J, bodies, M, t))
    assert lifted > 0  # the flag changes states the resolve would have lifted


def test_batched_simenv_custom_time_from_args(setup):
    """BatchedSimEnv built from the arg file with a custom reset window: the lanes' Philox reset
    times stay below time_max and their states equal the oracle's reset_state(t)."""
    amx, ens, ens_w, norms, args, J, bodies, M = setup
    ra = dict(RUN_PY_RESET_ARGS, custom_time=True, time_max=0.3)
    benv = amx.BatchedSimEnv(ens, None, lanes=256, deepmimic_args=args, reset_args=ra, seed=3, max_steps=2)
    e = benv.engine
    e.reset_all()
    e.num_steps.fill_(299)  # every lane reaches the horizon in the first step
    acts = torch.zeros(256, A, dtype=torch.float64, device=DEV)
    benv.step(acts)
    torch.cuda.synchronize()
    assert e.done[0].all()
    t = e.reset_times[0].cpu().numpy()
    assert (t >= 0).all() and (t < 0.3).all()
    got = e.obs[1].cpu().numpy()
    for b in range(0, 256, 37):
        assert _rel(got[b], DR.reset_state(J, bodies, M, float(t[b]))) <= 1e-10


def test_sample_points_custom_time_motion(setup):
    """sample_points on a BatchedSimEnv built from the arg file with custom_time / time_max:
    every trajectory j of worker i starts from reset_state(t), t = np_random(12345 +
    base_seed * i + j).uniform(0, time_max) (sim_env.py:132, 276) -- the env's window, not the
    clip length -- and with rng='device' every start time stays below time_max."""
    amx, ens, ens_w, norms, args, J, bodies, M = setup
    ra = dict(RUN_PY_RESET_ARGS, custom_time=True, time_max=0.35)
    benv = amx.BatchedSimEnv(ens, None, lanes=64, deepmimic_args=args, reset_args=ra, seed=3, horizon=6,
                             record_means=True)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100, init_log_std=-0.25)
    pol = amx.DevicePolicy(ens.ctx, pw, log_std)
    W, N, base = 2, 40, 4
    paths = amx.sample_points(benv, pol, num_to_collect=N, base_seed=base, num_workers=W)
    q = int(np.ceil(N / W))
    k = 0
    for i in range(W):
        tot, j = 0, 0
        while tot < q:
            j += 1
            t = R.gym_np_random(12345 + base * i + j).uniform(low=0, high=0.35)
            assert _rel(paths[k]["observations"][0], DR.reset_state(J, bodies, M, t)) <= 1e-10, (i, j)
            tot += len(paths[k]["rewards"])
            k += 1
    assert k == len(paths)
    dev_paths = amx.sample_points(benv, pol, num_to_collect=N, base_seed=base, num_workers=W, rng="device")
    eng = next(iter(benv.engine.__dict__["_sampler_engines"].values()))
    assert eng.reset_time_max == pytest.approx(0.35)
    assert len(dev_paths) > 0


def test_sample_points_with_reset_noise(setup):
    """sample_points with reset_args noise on (AddNoise on every motion reset, row a5; ADVICE
    r04): the paths' first observations are finite and perturbed away from the plain reset states
    of their (seeded) reset times, and the env's CURRENT noise setting reaches the sampler's cached
    engine -- after set_reset_noise(None) the same call starts every trajectory at the plain
    reset state again.  (With noise on the draws come from Philox(engine seed; lane, reset#), not
    from the trajectory seed: sampler.py documents that those paths depend on the lane count.)"""
    amx, ens, ens_w, norms, args, J, bodies, M = setup
    ra = dict(RUN_PY_RESET_ARGS, custom_time=True, time_max=0.35, noise_max=0.1, radian=0.2)
    benv = amx.BatchedSimEnv(ens, None, lanes=64, deepmimic_args=args, reset_args=ra, seed=3, horizon=6,
                             record_means=True)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100, init_log_std=-0.25)
    pol = amx.DevicePolicy(ens.ctx, pw, log_std)
    W, N, base = 2, 40, 4

    def starts(paths):
        q, k, out = int(np.ceil(N / W)), 0, []
        for i in range(W):
            tot, j = 0, 0
            while tot < q:
                j += 1
                t = R.gym_np_random(12345 + base * i + j).uniform(low=0, high=0.35)
                out.append(_rel(paths[k]["observations"][0], DR.reset_state(J, bodies, M, t)))
                tot += len(paths[k]["rewards"])
                k += 1
        assert k == len(paths)
        return np.array(out)

    noisy = amx.sample_points(benv, pol, num_to_collect=N, base_seed=base, num_workers=W)
    assert all(np.isfinite(p["observations"]).all() for p in noisy)
    d = starts(noisy)
    assert (d > 1e-3).mean() > 0.9, d  # perturbed (pose noise up to 0.1, root yaw up to 0.2 rad)
    benv.engine.set_reset_noise(None)
    plain = amx.sample_points(benv, pol, num_to_collect=N, base_seed=base, num_workers=W)
    assert starts(plain).max() <= 1e-10
