"""Generate the golden fixtures (tests/golden/*.npz) by running the REFERENCE Python.

Dev-container only: imports dhruvsreenivas/amp_extensions from /root/reference (read-only)
and records the outputs of its own hot-path code on small seeded inputs.  Skips cleanly
when /root/reference is absent (the GPU box never has it).  No reference source is copied:
the fixtures are data only (seeds, small inputs, outputs).

Stubs are installed ONLY for imports the path does not use or that are absent here:
  gym (registration, Env base, EzPickle, seeding.np_random — gym 0.26.1's published
  algorithm Generator(PCG64(SeedSequence(seed)))), tkinter.messagebox.NO and
  torch.utils.tensorboard.SummaryWriter (unused imports of milo/milo/dynamics.py:2,12), and
  DeepMimicEnv/ArgParser (imported by sim_env.py:2,8; SimEnv is built with object.__new__ and
  reset() is served by a stub core that returns reset-table row floor(t)).

Usage:  python tests/golden/make_golden.py            (writes tests/golden/*.npz, *.pt)
        python tests/golden/make_golden.py --only g13  (one fixture set)
"""
from __future__ import annotations

import math
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("AMX_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

S, A = 226, 28
HUMANOID_FALL = [0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 12, 13, 14]


def install_stubs():
    gym = types.ModuleType("gym")
    gym_envs = types.ModuleType("gym.envs")
    gym_reg = types.ModuleType("gym.envs.registration")
    gym_reg.register = lambda **kw: None
    gym_utils = types.ModuleType("gym.utils")
    gym_seeding = types.ModuleType("gym.utils.seeding")

    def np_random(seed=None):
        seq = np.random.SeedSequence(seed)
        return np.random.Generator(np.random.PCG64(seq)), seq.entropy

    gym_seeding.np_random = np_random

    class EzPickle:  # plain pickling (the real one re-runs __init__, which needs DeepMimicCore)
        def __init__(self, *a, **k):
            pass

    class Env:
        pass

    gym_spaces = types.ModuleType("gym.spaces")
    gym_spaces.Box = lambda *a, **k: None
    gym_utils.EzPickle = EzPickle
    gym_utils.seeding = gym_seeding
    gym.Env, gym.spaces, gym.utils, gym.envs = Env, gym_spaces, gym_utils, gym_envs
    gym_envs.registration = gym_reg
    for name, mod in [("gym", gym), ("gym.envs", gym_envs), ("gym.envs.registration", gym_reg),
                      ("gym.utils", gym_utils), ("gym.utils.seeding", gym_seeding), ("gym.spaces", gym_spaces)]:
        sys.modules[name] = mod

    tk = types.ModuleType("tkinter")
    tkm = types.ModuleType("tkinter.messagebox")
    tkm.NO = "no"
    tk.messagebox = tkm
    tk.E = "e"  # unused `from tkinter import E` of milo/milo/utils.py:1
    sys.modules["tkinter"], sys.modules["tkinter.messagebox"] = tk, tkm
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    sys.modules["torch.utils.tensorboard"] = tb

    dm = types.ModuleType("deepmimic")
    dm_env = types.ModuleType("deepmimic.env")
    dm_env_m = types.ModuleType("deepmimic.env.deepmimic_env")
    dm_env_m.DeepMimicEnv = object
    dm_util = types.ModuleType("deepmimic.util")
    dm_ap = types.ModuleType("deepmimic.util.arg_parser")
    dm_ap.ArgParser = object
    for name, mod in [("deepmimic", dm), ("deepmimic.env", dm_env), ("deepmimic.env.deepmimic_env", dm_env_m),
                      ("deepmimic.util", dm_util), ("deepmimic.util.arg_parser", dm_ap)]:
        sys.modules[name] = mod
    for p in ("milo", "gym-simenv", "mjrl"):
        sys.path.insert(0, os.path.join(REF, p))


class StubCore:
    """Stands in for DeepMimicEnv in SimEnv.reset: reset_time(time=t) selects row floor(t)."""

    def __init__(self, table):
        self.table = table
        self.row = 0
        self.rows = []

    def reset_time(self, time=0, **kw):
        self.row = int(math.floor(time))
        self.rows.append(self.row)

    def record_state(self, agent):
        return np.array(self.table[self.row], dtype=np.float64)

    def seed(self, seed):
        pass

    def get_vel_offset(self):
        return 136


def synthetic_offline(n, seed=0):
    """Synthetic humanoid-shaped offline set: s ~ 0.5 N(0,1), s[:,0] ~ U(0.8,0.95),
    a ~ N(0,1), s' = s + 0.01 N(0,1)."""
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


def make_simenv(SimEnv, ensemble, table, horizon=300, seed=1):
    env = object.__new__(SimEnv)
    env.deepmimic = StubCore(table)
    env.seed_env(seed)
    env.dynamic_ensemble = ensemble
    env.device = torch.device("cpu")
    env.enable_velocity_check = False
    env.horizon = horizon
    env.ob = None
    env.num_steps = 0
    env.agentID = 0
    env.state_size, env.action_size = S, A
    env.time_min, env.time_max = 0, table.shape[0]
    env.reset_dict = dict(time=0)
    env.record_vel_as_pos = False
    env.record_all_world = False      # humanoid3d_rot_ctrl.txt has no RecordAllWorld
    env.record_world_root_pos = False  # humanoid3d_rot_ctrl.txt:4
    env.record_world_root_rot = True
    env.sampling_rate = 1.0 / 30
    import json
    with open(os.path.join(REF, "deepmimic/deepmimic/data/characters/humanoid3d.txt")) as f:
        hj = json.load(f)
    env.body_defs = hj["BodyDefs"]
    env.pos_dim, env.rot_dim = 3, 6
    env.fall_contact_bodies = np.array(HUMANOID_FALL)
    env.fall_contact_bodies_offset = (env.pos_dim + env.rot_dim) * env.fall_contact_bodies + 1
    env.fall_contact_bodies_params = [[hj["BodyDefs"][i]["Param0"], hj["BodyDefs"][i]["Param1"],
                                       hj["BodyDefs"][i]["Param2"]] for i in HUMANOID_FALL]
    env.fall_contact_bodies_shapes = [hj["BodyDefs"][i]["Shape"] for i in HUMANOID_FALL]
    env.reset_counter = 0
    env.dynamics = ensemble.models[0]
    return env


def main(argv=()):
    if not os.path.isdir(os.path.join(REF, "milo")):
        print(f"[make_golden] {REF} not present: nothing to do")
        return 0
    install_stubs()
    torch.set_num_threads(1)
    if len(argv) == 2 and argv[0] == "--only":
        globals()[f"make_{argv[1]}"]()
        print("[make_golden] wrote", argv[1], "to", OUT)
        return 0
    from milo.datasets import AmpDataset
    from milo.dynamics import DynamicsEnsemble
    from milo.linear_cost import RBFLinearCost
    from milo.gail_cost import GAILCost
    from gym_simenv.envs.sim_env import SimEnv
    from mjrl.policies.gaussian_mlp import MLP

    # ---- G7 transformations ------------------------------------------------------------
    s, a, s2 = synthetic_offline(2048, seed=0)
    ds = AmpDataset(torch.from_numpy(s).float(), torch.from_numpy(a).float(), torch.from_numpy(s2).float())
    tr = ds.get_transformations()
    np.savez_compressed(os.path.join(OUT, "g7_transformations.npz"), n=2048, seed=0,
                        **{k: v.numpy() for k, v in zip(["mu_s", "sd_s", "mu_a", "sd_a", "mu_d", "sd_d"], tr)})

    for tag, hidden in (("h64", [64] * 4), ("h512", [512] * 4)):
        # ---- G1 ensemble forward + G4 discrepancy / threshold ---------------------------
        ens = DynamicsEnsemble(S, A, ds, None, num_models=4, hidden_sizes=hidden, dense_connect=True,
                               transform=True, base_seed=100)
        for m in ens.models:  # as load_ensemble does (dynamics.py:128-131)
            m.state_mean, m.state_scale, m.action_mean, m.action_scale, m.diff_mean, m.diff_scale = ens.transformations
        rs = np.random.RandomState(7)
        Bq = 64 if tag == "h64" else 16
        qs = torch.from_numpy(rs.randn(Bq, S) * 0.5).float()
        qa = torch.from_numpy(rs.randn(Bq, A)).float()
        preds = torch.stack([m.forward(qs, qa) for m in ens.models]).detach().numpy()
        disc = ens.get_action_discrepancy(qs, qa).numpy()
        ens.compute_threshold()
        np.savez_compressed(os.path.join(OUT, f"g1_ensemble_{tag}.npz"), hidden=np.array(hidden), base_seed=100,
                            query_seed=7, B=Bq, preds=preds, disc=disc, threshold=np.float64(ens.threshold),
                            first_w0=ens.models[0].model.fc_layers[0].weight.detach().numpy()[:4, :8])

    # ---- G2 SimEnv step traces (h64 ensemble), injected actions, with resets ---------------
    ens = DynamicsEnsemble(S, A, ds, None, num_models=4, hidden_sizes=[64] * 4, dense_connect=True,
                           transform=True, base_seed=100)
    for m in ens.models:
        m.state_mean, m.state_scale, m.action_mean, m.action_scale, m.diff_mean, m.diff_scale = ens.transformations
    table, _, _ = synthetic_offline(64, seed=1)
    env = make_simenv(SimEnv, ens, table, horizon=12, seed=5)
    rs = np.random.RandomState(2)
    T = 40
    acts = rs.randn(T, A) * math.exp(-0.25)
    obs, nobs, dones, model_idx, rows, nsteps = [], [], [], [], [], []
    o = env.reset()
    for t in range(T):
        model_idx.append(env.reset_counter)
        no, r, d, info = env.step(acts[t].copy())
        obs.append(o), nobs.append(no), dones.append(d), nsteps.append(env.num_steps)
        o = env.reset() if d else no
    np.savez_compressed(os.path.join(OUT, "g2_simenv_trace.npz"), table_seed=1, table_rows=64, horizon=12,
                        env_seed=5, actions=acts, obs=np.array(obs), next_obs=np.array(nobs),
                        done=np.array(dones), model_idx=np.array(model_idx), reset_rows=np.array(env.deepmimic.rows),
                        num_steps=np.array(nsteps))

    # ---- G3 fall-check boundary cases -------------------------------------------------------
    env = make_simenv(SimEnv, ens, table, horizon=300, seed=5)
    cases, results = [], []
    base = np.zeros(S)
    base[0] = 0.9
    for bi in range(len(HUMANOID_FALL)):
        off = env.fall_contact_bodies_offset[bi]
        radius = 0.5 * env.fall_contact_bodies_params[bi][0]
        thr = radius + 0.0001
        for delta in (-1, 0, 1):
            for ny in (0.0, 0.7, -1.0):
                ob = base.copy()
                if env.fall_contact_bodies_shapes[bi] == "capsule":
                    ob[off + 3 + 1] = ny
                    h = env.fall_contact_bodies_params[bi][1]
                    target = thr - (0.5 * h * ny if ny < 0 else -0.5 * h * ny)  # lower cap at thr
                else:
                    target = thr
                rel = target - ob[0]
                ob[off + 1] = rel
                ob[off + 1] = np.nextafter(rel, np.inf) if delta > 0 else (np.nextafter(rel, -np.inf) if delta < 0 else rel)
                env.ob = ob
                cases.append(ob.copy())
                results.append(env.check_collision())
    np.savez_compressed(os.path.join(OUT, "g3_fall_boundary.npz"), obs=np.array(cases), collided=np.array(results))

    # ---- G5 RFF MMD cost --------------------------------------------------------------------
    es, _, es2 = synthetic_offline(512, seed=3)
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], dim=1)
    cost = RBFLinearCost(expert, feature_dim=512, input_type="ss", bw_quantile=0.1, bw_samples=100000,
                         lambda_b=0.0025, seed=100)
    ps, pa, ps2 = synthetic_offline(96, seed=4)
    mb_mmd = cost.fit_cost(torch.cat([torch.from_numpy(ps), torch.from_numpy(ps2)], 1).float())
    ens.compute_threshold()
    bc, info = cost.get_bonus_costs(torch.from_numpy(ps).float(), torch.from_numpy(pa).float(), ens,
                                    next_states=torch.from_numpy(ps2).float())
    np.savez_compressed(os.path.join(OUT, "g5_rff_mmd.npz"), expert_seed=3, n_expert=512, pi_seed=4, n_pi=96,
                        feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100, bw=np.float64(cost.bw),
                        W_head=cost.rff.weight.detach().numpy()[:4, :8], b_head=cost.rff.bias.detach().numpy()[:8],
                        phi_e=cost.phi_e.numpy(), w=cost.w.numpy(), mb_mmd=np.float64(mb_mmd),
                        threshold=np.float64(ens.threshold), cost=bc.numpy(), ipm=info["ipm"].numpy(),
                        bonus=info["bonus"].numpy(), v_targ=info["v_targ"].numpy(),
                        expert_cost=np.float64(cost.get_expert_cost().item()))

    # ---- G6 GAIL / AMP LS discriminator -------------------------------------------------------
    for tag, hid in (("h64", [64, 32]), ("h1024", [1024, 512])):
        g = GAILCost(expert, agent_rb=None, feature_dim=1, hidden_dims=hid, input_type="ss", lambda_b=0.0025,
                     seed=100)
        ss = torch.cat([torch.from_numpy(ps), torch.from_numpy(ps2)], 1).float()
        c_plain = g.get_costs(ss)
        bc, info = g.get_bonus_costs(torch.from_numpy(ps).float(), torch.from_numpy(pa).float(), ens,
                                     next_states=torch.from_numpy(ps2).float())
        logits = g.disc(ss).detach()
        np.savez_compressed(os.path.join(OUT, f"g6_gail_{tag}.npz"), hidden=np.array(hid), seed=100,
                            lambda_b=0.0025, logits=logits.numpy(), cost_plain=c_plain.numpy(), cost=bc.numpy(),
                            ipm=info["ipm"].numpy(), bonus=info["bonus"].numpy())

    # ---- G8 2-worker sample_points with the stub reset core ----------------------------------
    from milo.sampler import sample_points
    pol = MLP(S, A, hidden_sizes=(32, 32), seed=100, init_log_std=-0.25, min_log_std=-2.0)
    pol_w = [(l.weight.detach().numpy(), l.bias.detach().numpy()) for l in pol.model.fc_layers]
    env = make_simenv(SimEnv, ens, table, horizon=8, seed=None)
    paths = sample_points(env, pol, num_to_collect=24, base_seed=100, num_workers=2, mode="samples",
                          deepmimic=False)
    np.savez_compressed(os.path.join(OUT, "g8_sample_points.npz"), horizon=8, num_to_collect=24, base_seed=100,
                        num_workers=2, lengths=np.array([len(p["rewards"]) for p in paths]),
                        observations=np.concatenate([p["observations"] for p in paths]),
                        next_observations=np.concatenate([p["next_observations"] for p in paths]),
                        actions=np.concatenate([p["actions"] for p in paths]),
                        means=np.concatenate([p["agent_infos"]["mean"] for p in paths]),
                        terminated=np.array([p["terminated"] for p in paths]),
                        pol_w0=pol_w[0][0][:4, :8])
    make_g9()
    make_g10()
    make_g11()
    make_g12()
    make_g13()
    print("[make_golden] wrote fixtures to", OUT)
    return 0


def g9_paths(seed=9):
    """Synthetic paths for G9: ragged lengths (incl. 1), observations beyond the +-10 clip,
    one path not terminated; float32 rewards as the relabel leaves them."""
    rs = np.random.RandomState(seed)
    lens = [1, 5, 17, 40, 3, 64, 2, 9]
    paths = []
    for i, l in enumerate(lens):
        obs = rs.randn(l, S) * 4.0
        obs[:, 3] *= 6.0  # some |x| > 10
        paths.append(dict(observations=obs, actions=np.zeros((l, A)), rewards=(rs.randn(l) * 0.3).astype(np.float32),
                          terminated=(i != 3)))
    return paths


def make_g9():
    """G9: returns / MLPBaseline / GAE / whitening (mjrl process_samples.py, mlp_baseline.py,
    batch_reinforce.py:271-297), run through the reference code.  The reference pins numpy
    1.21 (environment.yml), where a float32 scalar + Python float promotes to float64, so
    discount_sum accumulates in float64; numpy >= 2 here (NEP 50) would keep float32.  To
    record the pinned behaviour, discount_sum's input is widened to float64 (exact) before the
    reference loop runs, and process_paths sums path rewards as float64 for the same reason.
    Array-array arithmetic (the float32 deltas of non-terminated paths, whose b1 stays
    float32) promotes identically in both numpy versions and is left as is."""
    import copy
    import mjrl.utils.process_samples as ps
    from mjrl.algos.batch_reinforce import BatchREINFORCE
    from mjrl.baselines.mlp_baseline import MLPBaseline

    torch.manual_seed(500)
    bl = MLPBaseline(inp_dim=S, hidden_sizes=(128, 128))
    layers = [(m.weight.detach().numpy(), m.bias.detach().numpy()) for m in bl.model if isinstance(m, torch.nn.Linear)]
    paths = g9_paths()
    out = {}
    orig_discount_sum = ps.discount_sum
    ps.discount_sum = lambda x, gamma, terminal=0.0: orig_discount_sum(np.asarray(x, dtype=np.float64), gamma,
                                                                      terminal)
    for mode, lam in (("gae", 0.97), ("std", None)):
        pp = copy.deepcopy(paths)
        ps.compute_returns(pp, 0.995)
        ps.compute_advantages(pp, bl, 0.995, lam)
        out[f"returns_{mode}"] = np.concatenate([p["returns"] for p in pp])
        out[f"baseline_{mode}"] = np.concatenate([p["baseline"] for p in pp])
        out[f"adv_{mode}"] = np.concatenate([p["advantages"] for p in pp])
        if mode == "gae":
            stub = types.SimpleNamespace(running_score=None)
            pp64 = [dict(p, rewards=p["rewards"].astype(np.float64)) for p in pp]
            _, _, adv_w, base_stats, _ = BatchREINFORCE.process_paths(stub, pp64)
            out["adv_whitened"] = adv_w
            out["base_stats"] = np.array(base_stats, dtype=np.float64)
    feat = bl._features(paths).astype(np.float32)
    out["features_head"], out["features_time"] = feat[:, :8], feat[:, -4:]
    np.savez_compressed(os.path.join(OUT, "g9_gae.npz"), seed=9, baseline_seed=500, gamma=0.995, gae_lambda=0.97,
                        lengths=np.array([len(p["rewards"]) for p in paths]),
                        terminated=np.array([p["terminated"] for p in paths]),
                        observations=np.concatenate([p["observations"] for p in paths]),
                        rewards=np.concatenate([p["rewards"] for p in paths]),
                        w0_head=layers[0][0][:4, :8], w2=layers[2][0], **out)
    ps.discount_sum = orig_discount_sum


def g10_dbs(seed=10):
    """Synthetic trajectory databases in the reference's on-disk layout (collect_data.py /
    collect_expert.py): offline [{'episode': (states, actions, rewards), 'dtw_cost', 'ep_rew'}],
    expert [{'episode': states}], numpy arrays as the collectors save them."""
    rs = np.random.RandomState(seed)
    offline = []
    for T in (5, 1, 12, 7):
        offline.append({"episode": (rs.randn(T + 1, S), rs.randn(T, A).astype(np.float32), rs.randn(T)),
                        "dtw_cost": float(rs.rand()), "ep_rew": np.float64(rs.randn())})
    expert = [{"episode": rs.randn(T + 1, S)} for T in (4, 9, 2)]
    return offline, expert


def make_g10():
    """G10: milo/milo/utils.py get_db_mjrl / get_paths_mjrl / convert_to_veltopos on files
    written with torch.save, read back by the reference loaders (torch.load under an
    allow-list of numpy's reconstructors: torch >= 2.6 defaults to weights_only)."""
    import tempfile
    import milo.utils as U
    from amp_extensions_amd.datasets import _numpy_safe_globals

    offline, expert = g10_dbs()
    out = {}
    with tempfile.TemporaryDirectory() as d, torch.serialization.safe_globals(_numpy_safe_globals()):
        fo, fe = os.path.join(d, "offline.pt"), os.path.join(d, "expert.pt")
        torch.save(offline, fo)
        torch.save(expert, fe)
        for tag, kw in (("amp", dict(imitate_amp=True)), ("rew", dict(imitate_amp=False)),
                        ("n2", dict(num_trajs=2)), ("idx", dict(idx=2, num_trajs="all"))):
            if tag == "idx":
                continue  # utils.py:253 iterates the selected dict's keys (crashes): not recorded
            s_, a_, s2_ = U.get_db_mjrl(fo, **kw)
            out[f"db_{tag}_s"], out[f"db_{tag}_a"], out[f"db_{tag}_s2"] = s_.numpy(), a_.numpy(), s2_.numpy()
        es, es2 = U.get_db_mjrl(fe, expert=True)
        out["ex_s"], out["ex_s2"] = es.numpy(), es2.numpy()
        paths = U.get_paths_mjrl(fo, idx=1)
        out["paths_idx1_obs"], out["paths_idx1_act"] = paths[0]["observations"], paths[0]["actions"]
        paths = U.get_paths_mjrl(fe, expert=True)
        out["paths_ex_nobs"] = np.concatenate([p["next_observation"] for p in paths])

        class Core:
            def get_vel_offset(self):
                return 136

            def get_agent_update_rate(self):
                return 30

        x = U.convert_to_veltopos(fo, Core(), False, False)
        out["v2p_offline"] = np.concatenate([t["episode"][0] for t in x])
        x = U.convert_to_veltopos(fe, Core(), False, True)
        out["v2p_expert"] = np.concatenate([t["episode"] for t in x])
    np.savez_compressed(os.path.join(OUT, "g10_db.npz"), seed=10, **out)


def g11_paths(pol, seed=11):
    """Synthetic rollout for G11: float32-representable observations (the policy reads
    float32), actions = policy mean + exp(log_std) noise, raw advantages and rewards."""
    rs = np.random.RandomState(seed)
    paths = []
    for T in (7, 1, 30, 12, 50, 3, 25, 64):
        obs = (0.5 * rs.randn(T, S)).astype(np.float32).astype(np.float64)
        obs[:, 0] = rs.uniform(0.8, 0.95, T).astype(np.float32)
        mean = pol.model(torch.from_numpy(obs).float()).detach().numpy()
        act = mean.astype(np.float64) + np.exp(-0.25) * rs.randn(T, A)
        paths.append(dict(observations=obs, actions=act, advantages=rs.randn(T) * 2.0 + 0.3,
                          rewards=rs.randn(T)))
    return paths


def make_g11():
    """G11: one NPG policy update (mjrl/mjrl/algos/npg_cg.py:113-199: VPG gradient, Fisher
    HVP by double backward of mean_kl, 10-iteration CG, normalized step, set_param_values
    with the log_std clamp) on MILO's policy config (MLP(32,32), init_log_std -0.25,
    min_log_std -2, kl_dist 0.05 -> normalized_step_size 0.1, damping 1e-4), plus one HVP of
    a fixed vector."""
    from mjrl.algos.npg_cg import NPG
    from mjrl.policies.gaussian_mlp import MLP

    torch.set_num_threads(1)
    pol = MLP(S, A, hidden_sizes=(32, 32), seed=100, init_log_std=-0.25, min_log_std=-2.0)
    p0 = pol.get_param_values()
    paths = g11_paths(pol)
    agent = NPG(None, pol, None, normalized_step_size=0.1, FIM_invert_args={"iters": 10, "damping": 1e-4},
                hvp_sample_frac=1.0, seed=100, save_logs=False)
    obs, act, adv_w, _, _ = agent.process_paths(paths)
    v = np.random.RandomState(111).randn(p0.size).astype(np.float32)
    hvp = agent.HVP(obs, act, v)
    infos = {}
    agent.train_from_paths(paths, infos)
    p1 = pol.get_param_values()
    np.savez_compressed(os.path.join(OUT, "g11_npg.npz"), seed=11, step=0.1, damping=1e-4, cg_iters=10,
                        min_log_std=-2.0, lengths=np.array([len(p["advantages"]) for p in paths]),
                        observations=obs.astype(np.float32), actions=act,
                        advantages=np.concatenate([p["advantages"] for p in paths]), adv_whitened=adv_w,
                        params0=p0, hvp_v=v, hvp=hvp, vpg=infos["vpg_grad"], npg=infos["npg_grad"],
                        surr_before=np.float64(infos["surr_before"]), surr_after=np.float64(infos["surr_after"]),
                        params1=p1)



def make_g12():
    """G12: the data the reset-from-motion path reads — the humanoid3d character file and the
    spinkick clip (deepmimic/deepmimic/data/characters/humanoid3d.txt, data/motions/
    humanoid3d_spinkick.txt) as the reference holds them, so the GPU box (which has no
    /root/reference) can run the motion-reset tests.  Data only: the JSON text of the
    character and the clip's frame array.  No reference output exists for this path (the C++
    core is unbuildable here): the tests compare the device kernel with oracle/deepmimic_ref.py
    ("parity unpinned")."""
    base = os.path.join(REF, "deepmimic", "deepmimic", "data")
    with open(os.path.join(base, "characters", "humanoid3d.txt")) as f:
        character = f.read()
    import json
    motion = json.load(open(os.path.join(base, "motions", "humanoid3d_spinkick.txt")))
    ctrl = json.load(open(os.path.join(base, "controllers", "humanoid3d_rot_ctrl.txt")))
    np.savez_compressed(os.path.join(OUT, "g12_motion.npz"), character_json=np.array(character),
                        frames=np.array(motion["Frames"], dtype=np.float64), loop=np.array(motion["Loop"]),
                        record_world_root_pos=bool(ctrl.get("RecordWorldRootPos", False)),
                        record_world_root_rot=bool(ctrl.get("RecordWorldRootRot", False)),
                        record_all_world=bool(ctrl.get("RecordAllWorld", False)))


G13_HIDDEN = [32, 32]
# run.py's dynamics optimizer defaults (milo/milo/arguments.py:56-59: --dynamic_optim adam,
# --dynamic_lr 1e-3, --dynamic_eps 1e-8)
G13_OPTIM = {"optim": "adam", "lr": 1e-3, "eps": 1e-8}


def make_g13():
    """G13: the ensemble checkpoint run.py loads (run.py:63-78, 105, 108).  A reference
    DynamicsEnsemble (S/A 226/28, dense [32, 32] -- run.py's default depth -- Adam at run.py's
    defaults, base_seed 100) takes one optimizer step per member on the G7 offline set (so the
    weights are no longer the seed's and 'optim' holds Adam state), is written by the
    reference's own save_ensemble (a list of {'model', 'optim'}, dynamics.py:110-116) to
    g13_ensemble.pt, then loaded back into a fresh reference ensemble exactly as run.py:72-78
    does, followed by compute_threshold() (run.py:108).  Recorded: the threshold, every
    member's forward (un-normalised and normalised) and the disagreement on seeded query rows."""
    from milo.datasets import AmpDataset
    from milo.dynamics import DynamicsEnsemble

    s, a, s2 = synthetic_offline(2048, seed=0)
    ds = AmpDataset(torch.from_numpy(s).float(), torch.from_numpy(a).float(), torch.from_numpy(s2).float())
    kw = dict(num_models=4, batch_size=256, hidden_sizes=G13_HIDDEN, transform=True, dense_connect=True,
              optim_args=G13_OPTIM, base_seed=100, device=torch.device("cpu"))
    ens = DynamicsEnsemble(S, A, ds, None, **kw)
    for m in ens.models:  # as DynamicsModel.train sets them (dynamics.py:311-313)
        m.state_mean, m.state_scale, m.action_mean, m.action_scale, m.diff_mean, m.diff_scale = ens.transformations
    rs = np.random.RandomState(13)
    idx = rs.permutation(2048)[:256]
    for m in ens.models:
        m.train_step(0, ds.states[idx], ds.actions[idx], ds.next_states[idx])
    path = os.path.join(OUT, "g13_ensemble.pt")
    ens.save_ensemble(path)
    # run.py:72-78 + 108 as written
    loaded = DynamicsEnsemble(S, A, ds, None, **kw)
    loaded.load_ensemble(path)
    loaded.compute_threshold()
    qs = torch.from_numpy(rs.randn(48, S) * 0.5).float()
    qs[:, 0] = torch.from_numpy(rs.uniform(0.8, 0.95, 48)).float()
    qa = torch.from_numpy(rs.randn(48, A)).float()
    with torch.no_grad():
        preds = torch.stack([m.forward(qs, qa) for m in loaded.models]).numpy()
        preds_norm = torch.stack([m.forward(qs, qa, unnormalize_out=False) for m in loaded.models]).numpy()
    disc = loaded.get_action_discrepancy(qs, qa).numpy()
    np.savez_compressed(os.path.join(OUT, "g13_ensemble_ckpt.npz"), hidden=np.array(G13_HIDDEN), base_seed=100,
                        offline_seed=0, n_offline=2048, optim="adam", lr=1e-3, eps=1e-8, query_s=qs.numpy(),
                        query_a=qa.numpy(), preds=preds, preds_norm=preds_norm, disc=disc,
                        threshold=np.float64(loaded.threshold))


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
