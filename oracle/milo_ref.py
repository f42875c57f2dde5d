"""CPU restatement of the reference rollout hot path (TEST INFRASTRUCTURE ONLY).

Each function restates one reference routine (paths relative to the reference root) with
the same floating-point operation order, so that on the same inputs it reproduces the
reference's numbers: bit-for-bit where the reference is numpy/torch-CPU code run on the
same machine (checked against tests/golden/*.npz), and as the CPU comparator for the HIP
engine elsewhere.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# normalizers — milo/milo/datasets.py:23-43 (AmpDataset.get_transformations)
# --------------------------------------------------------------------------------------


def get_transformations(states: torch.Tensor, actions: torch.Tensor, next_states: torch.Tensor):
    """(mu_s, sd_s, mu_a, sd_a, mu_d, sd_d): column means and mean-absolute-deviation
    + 1e-8 (not the std) of s, a and s'-s (datasets.py:27-43)."""
    diff = next_states - states
    state_mean = states.mean(dim=0).float()
    action_mean = actions.mean(dim=0).float()
    diff_mean = diff.mean(dim=0).float()
    state_scale = torch.abs(states - state_mean).mean(dim=0).float() + 1e-8
    action_scale = torch.abs(actions - action_mean).mean(dim=0).float() + 1e-8
    diff_scale = torch.abs(diff - diff_mean).mean(dim=0).float() + 1e-8
    return state_mean, state_scale, action_mean, action_scale, diff_mean, diff_scale


# --------------------------------------------------------------------------------------
# dense-connect MLP ensemble — milo/milo/dynamics.py:167-233, 394-433
# --------------------------------------------------------------------------------------


def basic_mlp_layer_shapes(S: int, A: int, hidden: list[int]) -> list[tuple[int, int]]:
    """(out, in) of every nn.Linear of BasicMLP(S+A -> S, hidden, dense_connect=True),
    dynamics.py:412-420: layer i takes the concat of every previous layer's width."""
    sizes = [S + A] + list(hidden) + [S]
    shapes = []
    for i in range(len(sizes) - 1):
        fan_in = sizes[i] + sum(sizes[:i])
        shapes.append((sizes[i + 1], fan_in))
    return shapes


def init_model_weights(S: int, A: int, hidden: list[int], seed: int) -> list[tuple[torch.Tensor, torch.Tensor]]:
    """Weights of one ensemble member exactly as DynamicsModel.__init__ draws them:
    torch.manual_seed(seed); np.random.seed(seed) (dynamics.py:185-186), then the
    nn.Linear layers of BasicMLP constructed in order (default kaiming-uniform weight +
    uniform bias, dynamics.py:419)."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    out = []
    for (o, i) in basic_mlp_layer_shapes(S, A, hidden):
        lin = nn.Linear(i, o)
        out.append((lin.weight.detach().clone(), lin.bias.detach().clone()))
    return out


def init_ensemble_weights(S: int, A: int, hidden: list[int], num_models: int = 4, base_seed: int = 100):
    """DynamicsEnsemble.__init__: member k seeded base_seed + k (dynamics.py:70-79)."""
    return [init_model_weights(S, A, hidden, base_seed + k) for k in range(num_models)]


def basic_mlp_forward(weights, x: torch.Tensor) -> torch.Tensor:
    """BasicMLP.forward with dense_connect and ReLU (dynamics.py:422-433)."""
    inp = x
    for (W, b) in weights[:-1]:
        out = torch.relu(F.linear(inp, W, b))
        inp = torch.cat([inp, out], dim=1)
    W, b = weights[-1]
    return F.linear(inp, W, b)


def dynamics_forward(weights, norms, state: torch.Tensor, action: torch.Tensor, unnormalize_out: bool = True):
    """DynamicsModel.forward with transform=True (dynamics.py:216-233)."""
    mu_s, sd_s, mu_a, sd_a, mu_d, sd_d = norms
    s = (state - mu_s) / sd_s
    a = (action - mu_a) / sd_a
    y = basic_mlp_forward(weights, torch.cat([s, a], dim=1))
    if unnormalize_out:
        y = (y * sd_d) + mu_d
    return y


def compute_discrepancy(ens_weights, norms, state: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
    """DynamicsEnsemble.compute_discrepancy (dynamics.py:134-143): max over model pairs
    (i<j) of ||pred_i - pred_j||_2 over the state dimension."""
    with torch.no_grad():
        preds = torch.cat([dynamics_forward(w, norms, state, action).unsqueeze(0) for w in ens_weights], dim=0)
    disc = torch.cat([torch.norm(preds[i] - preds[j], p=2, dim=1).unsqueeze(0)
                      for i in range(preds.shape[0]) for j in range(i + 1, preds.shape[0])], dim=0)
    return disc.max(0).values


def ensemble_preds(ens_weights, norms, state: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
    with torch.no_grad():
        return torch.stack([dynamics_forward(w, norms, state, action) for w in ens_weights], dim=0)


def load_ensemble_weights(path) -> list:
    """DynamicsEnsemble.load_ensemble (dynamics.py:118-126) reduced to what the forward needs:
    the list of {'model', 'optim'} dicts save_ensemble writes (dynamics.py:110-116), each
    member's BasicMLP state dict ('fc_layers.{i}.weight/bias') as [(W, b), ...].  Read with the
    weights-only unpickler."""
    sds = torch.load(path, map_location="cpu", weights_only=True)
    out = []
    for sd in sds:
        m = sd["model"]
        n = 1 + max(int(k.split(".")[1]) for k in m if k.startswith("fc_layers."))
        out.append([(m[f"fc_layers.{i}.weight"], m[f"fc_layers.{i}.bias"]) for i in range(n)])
    return out


def compute_threshold(ens_weights, norms, states: torch.Tensor, actions: torch.Tensor, batch_size: int = 256) -> float:
    """compute_threshold (dynamics.py:145-152): max discrepancy over the offline set.
    The reference iterates a shuffled DataLoader; the max is order-independent."""
    res = [compute_discrepancy(ens_weights, norms, states[i:i + batch_size], actions[i:i + batch_size])
           for i in range(0, states.shape[0], batch_size)]
    return torch.cat(res, dim=0).max().item()


# --------------------------------------------------------------------------------------
# SimEnv step / termination — gym-simenv/gym_simenv/envs/sim_env.py
# --------------------------------------------------------------------------------------

# humanoid3d BodyDefs (deepmimic/deepmimic/data/characters/humanoid3d.txt) for the fall
# bodies of run_amp_humanoid3d_spinkick_args.txt:19 / sim_env.py:102
FALL_BODIES = [0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 12, 13, 14]
BODY_DEFS = {  # id: (shape, Param0, Param1)
    0: ("sphere", 0.18, 0.18), 1: ("sphere", 0.22, 0.22), 2: ("sphere", 0.205, 0.205),
    3: ("capsule", 0.11, 0.3), 4: ("capsule", 0.1, 0.31), 5: ("box", 0.177, 0.055),
    6: ("capsule", 0.09, 0.18), 7: ("capsule", 0.08, 0.135), 8: ("sphere", 0.08, 0.08),
    9: ("capsule", 0.11, 0.3), 10: ("capsule", 0.1, 0.31), 11: ("box", 0.177, 0.055),
    12: ("capsule", 0.09, 0.18), 13: ("capsule", 0.08, 0.135), 14: ("sphere", 0.08, 0.08),
}


class SimEnvRef:
    """Restatement of SimEnv.step/is_done/check_*/reset (sim_env.py:140-285) with the
    DeepMimicCore reset replaced by an explicit reset-state row."""

    def __init__(self, ens_weights, norms, horizon=300, enable_velocity_check=False, record_all_world=False,
                 record_world_root_pos=False, record_vel_as_pos=False, sampling_rate=1.0 / 30, vel_offset=136,
                 fall_bodies=FALL_BODIES, body_defs=BODY_DEFS, pos_dim=3, rot_dim=6):
        self.ens = ens_weights
        self.norms = norms
        self.horizon = horizon
        self.enable_velocity_check = enable_velocity_check
        self.record_all_world = record_all_world
        self.record_world_root_pos = record_world_root_pos
        self.record_vel_as_pos = record_vel_as_pos
        self.sampling_rate = sampling_rate
        self.vel_offset = vel_offset
        self.pos_dim, self.rot_dim = pos_dim, rot_dim
        self.fall_contact_bodies = np.array(fall_bodies)
        self.fall_contact_bodies_offset = (pos_dim + rot_dim) * self.fall_contact_bodies + 1  # :103-104
        self.fall_contact_bodies_params = [[body_defs[i][1], body_defs[i][2]] for i in fall_bodies]
        self.fall_contact_bodies_shapes = [body_defs[i][0] for i in fall_bodies]
        self.ob = None
        self.num_steps = 0
        self.reset_counter = 0  # :118
        self.model_index = 0    # :119 models[0] until the first reset

    # sim_env.py:140-162
    def step(self, action: np.ndarray):
        assert self.ob is not None
        self.num_steps += 1
        with torch.no_grad():
            s = torch.from_numpy(self.ob).float().unsqueeze(0)
            a = torch.from_numpy(action).float().unsqueeze(0)
            d = dynamics_forward(self.ens[self.model_index], self.norms, s, a)
        self.ob += d.squeeze(0).numpy()
        done = self.is_done()
        return self.ob.copy(), 0, done, {}

    # :164-173
    def is_done(self) -> bool:
        horizon_done = self.num_steps >= self.horizon
        collided = self.check_collision()
        velocity_exploded = self.check_velocity() if self.enable_velocity_check else False
        return bool(horizon_done or collided or velocity_exploded)

    def _body_world_y(self, index: int, offset: int) -> float:
        if self.record_all_world or (index == 0 and self.record_world_root_pos):  # :181, :223
            return self.ob[offset + 1]
        return self.ob[0] + self.ob[offset + 1]

    # :175-189
    def check_sphere(self, index: int) -> bool:
        offset = self.fall_contact_bodies_offset[index]
        y = self._body_world_y(index, offset)
        radius = 0.5 * self.fall_contact_bodies_params[index][0]
        return bool(y <= radius + 0.0001)

    # :191-236
    def check_capsule(self, index: int) -> bool:
        offset = self.fall_contact_bodies_offset[index]
        radius = 0.5 * self.fall_contact_bodies_params[index][0]
        h = self.fall_contact_bodies_params[index][1]
        norm_y = self.ob[offset + self.pos_dim + 1]
        top = 0.5 * h * norm_y
        bottom = -0.5 * h * norm_y
        y = self._body_world_y(index, offset)
        return bool(y + top <= radius + 0.0001 or y + bottom <= radius + 0.0001)

    # :246-257
    def check_collision(self) -> bool:
        collided = False
        for i in range(len(self.fall_contact_bodies)):
            if self.fall_contact_bodies_shapes[i] == "sphere":
                collided |= self.check_sphere(i)
            elif self.fall_contact_bodies_shapes[i] == "capsule":
                collided |= self.check_capsule(i)
        return collided

    # :259-268 (in-place /= on the view mutates ob when RecordVelAsPos — kept)
    def check_velocity(self, threshold=100) -> bool:
        velocity = self.ob[self.vel_offset:]
        if self.record_vel_as_pos:
            velocity /= self.sampling_rate
        return bool(np.any(np.abs(velocity) > threshold))

    # :270-285 with the DeepMimicCore pose replaced by `row`
    def reset(self, row: np.ndarray) -> np.ndarray:
        self.num_steps = 0
        self.ob = np.array(row, dtype=np.float64, copy=True)
        self.reset_counter = (self.reset_counter + 1) % len(self.ens)
        self.model_index = self.reset_counter
        return self.ob.copy()


def step_update_terminate(ob: np.ndarray, pred_k: np.ndarray, num_steps: np.ndarray, horizon: int = 300,
                          **env_kw):
    """Vectorised-by-loop restatement used to check the HIP step kernel bit-for-bit:
    ob [B,S] f64, pred_k [B,S] f32 (already model-selected), num_steps [B] -> (ob', done, num_steps')."""
    env = SimEnvRef([None], None, horizon=horizon, **env_kw)
    B = ob.shape[0]
    out = np.empty_like(ob)
    done = np.zeros(B, dtype=np.uint8)
    ns = num_steps.astype(np.int32) + 1
    for b in range(B):
        env.ob = ob[b].copy()
        env.ob += pred_k[b].astype(np.float32)  # float32 -> float64 add (sim_env.py:158)
        env.num_steps = int(ns[b])
        done[b] = env.is_done()
        out[b] = env.ob
    return out, done, ns


# --------------------------------------------------------------------------------------
# MILO RFF MMD cost — milo/milo/linear_cost.py:6-152
# --------------------------------------------------------------------------------------


def cost_input(input_type: str, states, actions, next_states):
    """The cost-input row of a transition by input type: linear_cost.py:115-127,
    gail_cost.py:258-268 ('sa', 'ss', 'sas', 's'); batch_reinforce.py:107-110 builds the
    fit_cost input the same way."""
    if input_type == "sa":
        return torch.cat([states, actions], dim=1)
    if input_type == "ss":
        assert next_states is not None
        return torch.cat([states, next_states], dim=1)
    if input_type == "sas":
        return torch.cat([states, actions, next_states], dim=1)
    if input_type == "s":
        return states
    raise NotImplementedError("Input type not implemented")


class RBFLinearCostRef:
    """Restatement of RBFLinearCost (linear_cost.py:23-152), CPU torch."""

    def __init__(self, expert_data: torch.Tensor, feature_dim=1024, input_type="ss", cost_range=(-1.0, 0.0),
                 bw_quantile=0.1, bw_samples=100000, lambda_b=1.0, lr=0.0, seed=100):
        torch.manual_seed(seed)
        np.random.seed(seed)
        self.expert_data = expert_data
        input_dim = expert_data.size(1)
        self.input_type = input_type
        self.feature_dim = feature_dim
        self.cost_range = cost_range
        if cost_range is not None:
            self.c_min, self.c_max = cost_range
        self.lambda_b = lambda_b
        self.quantile = bw_quantile
        self.bw_samples = bw_samples
        self.bw = self.fit_bandwidth(expert_data)  # :50
        rff = nn.Linear(input_dim, feature_dim)     # :53 (consumes the RNG)
        rff.bias.data = (torch.rand_like(rff.bias.data) - 0.5) * 2.0 * np.pi  # :54
        rff.weight.data = torch.rand_like(rff.weight.data) / (self.bw + 1e-8)  # :55
        self.W = rff.weight.data
        self.b = rff.bias.data
        self.w = None
        self.expert_rep = self.get_rep(expert_data)  # :61
        self.phi_e = self.expert_rep.mean(dim=0)    # :62

    def get_rep(self, x):  # :64-71
        with torch.no_grad():
            out = F.linear(x.cpu(), self.W, self.b)
            return torch.cos(out) * np.sqrt(2 / self.feature_dim)

    def fit_bandwidth(self, data):  # :73-82
        n = data.shape[0]
        i0 = torch.randint(low=0, high=n, size=(self.bw_samples,))
        i1 = torch.randint(low=0, high=n, size=(self.bw_samples,))
        norm = torch.norm(data[i0, :] - data[i1, :], dim=1)
        return torch.quantile(norm, q=self.quantile).item()

    def fit_cost(self, data_pi):  # :84-94
        phi = self.get_rep(data_pi).mean(0)
        feat_diff = phi - self.phi_e
        self.w = feat_diff
        return torch.dot(self.w, feat_diff).item()

    def get_costs(self, x):  # :96-103
        data = self.get_rep(x)
        if self.cost_range is not None:
            return torch.clamp(torch.mm(data, self.w.unsqueeze(1)), self.c_min, self.c_max)
        return torch.mm(data, self.w.unsqueeze(1))

    def get_expert_cost(self):  # :105-109
        return (1 - self.lambda_b) * torch.clamp(torch.mm(self.expert_rep, self.w.unsqueeze(1)),
                                                 self.c_min, self.c_max).mean()

    def get_bonus_costs(self, states, actions, disc_fn, thr, next_states=None):  # :111-152
        """`disc_fn(states, actions)` is the ensemble's get_action_discrepancy."""
        rff_input = cost_input(self.input_type, states, actions, next_states)   # :115-127
        rff_cost = self.get_costs(rff_input)
        if self.cost_range is not None:                                          # :131-137
            discrepancy = disc_fn(states, actions) / thr
            discrepancy = discrepancy.view(-1, 1)
            discrepancy[discrepancy > 1.0] = 1.0
            bonus = discrepancy * self.c_min
        else:                                                                    # :138-139
            bonus = disc_fn(states, actions).view(-1, 1)
        ipm = (1 - self.lambda_b) * rff_cost
        weighted_bonus = self.lambda_b * bonus.cpu()
        cost = ipm - weighted_bonus
        return cost, {"bonus": weighted_bonus, "ipm": ipm, "v_targ": rff_cost, "cost": cost}


# --------------------------------------------------------------------------------------
# AMP / GAIL least-squares discriminator — milo/milo/gail_cost.py
# --------------------------------------------------------------------------------------


def init_disc_weights(input_dim: int, hidden=(1024, 512), output_dim=1, seed=100):
    """GAILCost.__init__ (gail_cost.py:60-83): torch/np seeded, Discriminator layers built
    in order (Linear(in,h0), Linear(h0,h1), Linear(h1,1), default init), then
    disc_weight_init applied in module order: xavier_uniform on every weight except the
    1-output layer, which gets U(-1, 1) (gail_cost.py:11-16, 39).  Biases keep the default."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    sizes = [input_dim] + list(hidden) + [output_dim]
    layers = [nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)]
    for lin in layers:
        if lin.out_features == 1:
            nn.init.uniform_(lin.weight.data, a=-1.0, b=1.0)
        else:
            nn.init.xavier_uniform_(lin.weight.data)
    return [(l.weight.detach().clone(), l.bias.detach().clone()) for l in layers]


def disc_forward(weights, x):
    """Discriminator.forward: Linear, ReLU, ..., Linear (gail_cost.py:28-42)."""
    h = x
    for i, (W, b) in enumerate(weights):
        h = F.linear(h, W, b)
        if i < len(weights) - 1:
            h = torch.relu(h)
    return h


def gail_ls_costs(weights, ss):
    """get_ls_costs (gail_cost.py:231-236)."""
    with torch.no_grad():
        d = disc_forward(weights, ss)
        rewards = 1.0 - 0.25 * (1.0 - d) ** 2
        rewards[rewards < 0.0] = 0.0
        return -rewards


def gail_ll_costs(weights, ss):
    """get_ll_costs (gail_cost.py:238-243): logsigmoid of the discriminator output."""
    with torch.no_grad():
        return F.logsigmoid(disc_forward(weights, ss))


def gail_bonus_costs(weights, states, actions, next_states, disc_fn, lambda_b, input_type="ss",
                     disc_loss_type="least_squares"):
    """get_bonus_costs (gail_cost.py:254-279); get_costs picks the loss type (:246-251)."""
    with torch.no_grad():
        inp = cost_input(input_type, states, actions, next_states)
        costs = gail_ls_costs if disc_loss_type == "least_squares" else gail_ll_costs
        input_cost = costs(weights, inp)
        ipm = (1 - lambda_b) * input_cost
        discrepancy = disc_fn(states, actions)
        bonus = lambda_b * discrepancy.view(-1, 1)
        cost = ipm - bonus
        return cost, {"bonus": bonus, "ipm": ipm, "v_targ": input_cost, "cost": cost}


# --------------------------------------------------------------------------------------
# Gaussian MLP policy — mjrl/mjrl/policies/gaussian_mlp.py, mjrl/mjrl/utils/fc_network.py
# --------------------------------------------------------------------------------------


def init_policy_weights(S: int, A: int, hidden=(32, 32), seed=100, init_log_std=-0.25):
    """MLP.__init__ (gaussian_mlp.py:28-40): seeded, FCNetwork layers in order, last
    layer's weight and bias scaled by 1e-2; log_std = init_log_std."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    sizes = (S,) + tuple(hidden) + (A,)
    layers = [nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)]
    layers[-1].weight.data = 1e-2 * layers[-1].weight.data
    layers[-1].bias.data = 1e-2 * layers[-1].bias.data
    log_std = torch.ones(A) * init_log_std
    return [(l.weight.detach().clone(), l.bias.detach().clone()) for l in layers], log_std


def policy_mean(pweights, ob: np.ndarray) -> np.ndarray:
    """FCNetwork.forward with identity in/out transforms (fc_network.py:42-55)."""
    o = torch.from_numpy(np.float32(ob.reshape(1, -1)))
    out = (o - torch.zeros(o.shape[1])) / (torch.ones(o.shape[1]) + 1e-8)
    for i, (W, b) in enumerate(pweights):
        out = F.linear(out, W, b)
        if i < len(pweights) - 1:
            out = torch.tanh(out)
    return out.detach().numpy().ravel()


def policy_action(pweights, log_std, ob: np.ndarray, noise: np.ndarray | None = None):
    """MLP.get_action (gaussian_mlp.py:95-104) with eps = 0; `noise` replaces
    np.random.randn(m) when given."""
    mean = policy_mean(pweights, ob)
    log_std_val = np.float64(log_std.numpy().ravel())
    if noise is None:
        np.random.uniform()  # the eps-greedy draw happens even at eps = 0 (gaussian_mlp.py:99)
        n = np.random.randn(mean.shape[0])
    else:
        n = noise
    act = mean + np.exp(log_std_val) * n
    return act, {"mean": mean, "log_std": log_std_val, "evaluation": mean}


# --------------------------------------------------------------------------------------
# Philox4x32-10 — the engine's device RNG (not part of the reference; restated here so
# reset-row choice and policy noise are checked bit-for-bit)
# --------------------------------------------------------------------------------------

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
TAG_RESET = 0x52534554
TAG_POLICY = 0x504F4C49


def philox4x32_10(ctr: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """ctr [..., 4] uint32, key (k0, k1) -> [..., 4] uint32 (Salmon et al. 2011)."""
    c = [ctr[..., i].astype(np.uint64) for i in range(4)]
    k0, k1 = np.uint32(key[0]), np.uint32(key[1])
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = _M0 * c[0]
        p1 = _M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return np.stack([x.astype(np.uint32) for x in c], axis=-1)


def u53(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return ((a >> np.uint32(5)).astype(np.float64) * 67108864.0 + (b >> np.uint32(6)).astype(np.float64)) * (
        1.0 / 9007199254740992.0)


def reset_rows(seed: int, lanes: np.ndarray, reset_count: np.ndarray, R: int) -> np.ndarray:
    """Row the engine's reset kernel picks for lane b on its reset_count-th reset."""
    ctr = np.stack([lanes.astype(np.uint32), reset_count.astype(np.uint32), np.zeros_like(lanes, np.uint32),
                    np.full(lanes.shape, TAG_RESET, np.uint32)], axis=-1)
    r = philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    x = (r[..., 1].astype(np.uint64) << np.uint64(32)) | r[..., 0].astype(np.uint64)
    return (x % np.uint64(R)).astype(np.int64)


def policy_noise(seed: int, counter: int, B: int, A: int) -> np.ndarray:
    """N(0,1) fp64 noise [B, A] of the engine's policy kernel (Box-Muller on one Philox
    block per action pair)."""
    lanes = np.arange(B, dtype=np.uint32)[:, None]
    pairs = np.arange((A + 1) // 2, dtype=np.uint32)[None, :]
    ctr = np.stack(np.broadcast_arrays(lanes, np.uint32(counter & 0xFFFFFFFF),
                                       (pairs << np.uint32(8)) | np.uint32((counter >> 32) & 0xFF),
                                       np.uint32(TAG_POLICY)), axis=-1).astype(np.uint32)
    r = philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    u1 = 1.0 - u53(r[..., 0], r[..., 1])
    u2 = u53(r[..., 2], r[..., 3])
    rad = np.sqrt(-2.0 * np.log(u1))
    ang = 6.283185307179586 * u2
    z = np.empty((B, 2 * pairs.shape[1]), np.float64)
    z[:, 0::2] = rad * np.cos(ang)
    z[:, 1::2] = rad * np.sin(ang)
    return z[:, :A]


# --------------------------------------------------------------------------------------
# relabel block — mjrl/mjrl/algos/batch_reinforce.py:103-169 (MMD branch with ensemble)
# --------------------------------------------------------------------------------------


def relabel_mmd(paths, cost: RBFLinearCostRef, disc_fn, thr):
    """Replaces traj['rewards'] with -bonus_cost per path and returns infos."""
    infos = {"int": [], "ext": [], "reward": [], "ep_len": []}
    cost_input = np.concatenate([np.concatenate([p["observations"], p["next_observations"]], axis=1)
                                 for p in paths], axis=0)
    infos["mb_mmd"] = cost.fit_cost(torch.from_numpy(cost_input).float())
    for traj in paths:
        s = torch.from_numpy(traj["observations"]).float()
        s2 = torch.from_numpy(traj["next_observations"]).float()
        a = torch.from_numpy(traj["actions"]).float()
        bonus_cost, ci = cost.get_bonus_costs(s, a, disc_fn, thr, next_states=s2)
        bonus_cost = bonus_cost[:, 0]
        isum = -np.sum(ci["bonus"][:, 0].numpy())
        esum = -np.sum(ci["ipm"][:, 0].numpy())
        infos["int"].append(isum)
        infos["ext"].append(esum)
        infos["reward"].append(esum + isum)
        infos["ep_len"].append(len(traj["rewards"]))
        traj["rewards"] = -1.0 * bonus_cost.cpu().numpy()
    infos["bonus_mmd"] = np.concatenate([-1.0 * t["rewards"] for t in paths], axis=0).mean() - \
        cost.get_expert_cost()
    return infos


# --------------------------------------------------------------------------------------
# sampler — milo/milo/sampler.py:8-151 (restated for the CPU baseline and path checks)
# --------------------------------------------------------------------------------------


def stack_tensor_dict_list(lst):
    """sampler.py:133-151."""
    ret = {}
    for k in lst[0].keys():
        ex = lst[0][k]
        ret[k] = stack_tensor_dict_list([x[k] for x in lst]) if isinstance(ex, dict) else np.array([x[k] for x in lst])
    return ret


def gym_np_random(seed: int) -> np.random.Generator:
    """gym 0.26.1 gym.utils.seeding.np_random (the pinned gym of environment.yml:123):
    Generator(PCG64(SeedSequence(seed)))."""
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


def get_samples(env: SimEnvRef, pweights, log_std, num_to_collect: int, seed: int, reset_table: np.ndarray,
                mode="samples", eval_mode=False, time_max=None):
    """get_samples (sampler.py:8-84) with env.reset's motion time t = np_random.uniform(0, time_max)
    (sim_env.py:276; time_max = the table's R rows, or reset_args['time_max'] with custom_time,
    sim_env.py:76-77) selecting row floor(t) of the reset table in place of the DeepMimicCore
    pose.  A missing info['valid'] is treated as valid (SimEnv returns {})."""
    paths, samples, ctr_seed = [], 0, 0
    cond = (lambda: len(paths) < num_to_collect) if mode == "trajectories" else (lambda: samples < num_to_collect)
    while cond():
        ctr_seed += 1
        rng = gym_np_random(seed + ctr_seed)             # env.seed_env(seed + ctr), sim_env.py:132
        np.random.seed(seed + ctr_seed)                   # sampler.py:39
        row = int(rng.uniform(low=0, high=reset_table.shape[0] if time_max is None else time_max))
        o = env.reset(reset_table[row])
        obs, nobs, acts, rews, ainfos, einfos = [], [], [], [], [], []
        done = False
        while not done:
            a, ai = policy_action(pweights, log_std, o)
            a = ai["evaluation"] if eval_mode else a
            no, r, done, info = env.step(a)
            obs.append(o); nobs.append(no); acts.append(a); rews.append(r); ainfos.append(ai); einfos.append(info)
            o = no
        paths.append(dict(observations=np.array(obs), next_observations=np.array(nobs), actions=np.array(acts),
                          rewards=np.array(rews), agent_infos=stack_tensor_dict_list(ainfos), env_infos=einfos,
                          terminated=done))
        samples += len(obs)
    return paths, samples


def _worker(args):
    torch.set_num_threads(1)
    (ens, norms, pweights, log_std, quota, seed, table, env_kw) = args
    env = SimEnvRef(ens, norms, **env_kw)
    return get_samples(env, pweights, log_std, quota, seed, table)


def sample_points(ens, norms, pweights, log_std, num_to_collect: int, base_seed: int, reset_table, num_workers=4,
                  env_kw=None, pool=None):
    """sample_points (sampler.py:87-130): quota ceil(N/W) per worker, seeds 12345 + base_seed*i."""
    per = math.ceil(num_to_collect / num_workers)
    args = [(ens, norms, pweights, log_std, per, 12345 + base_seed * i, reset_table, env_kw or {})
            for i in range(num_workers)]
    if pool is None:
        results = [_worker(a) for a in args]
    else:
        results = pool.map(_worker, args)
    paths = []
    for p, _ in results:
        paths.extend(p)
    return paths


# --------------------------------------------------------------------------------------
# returns / MLP value baseline / GAE — mjrl/mjrl/utils/process_samples.py:3-45,
# mjrl/mjrl/baselines/mlp_baseline.py:10-108, mjrl/mjrl/algos/batch_reinforce.py:271-297
# Promotion follows the reference's pinned numpy 1.21 (environment.yml): scalar float32 +
# Python float -> float64, so discount_sum accumulates in float64 (its input is widened up
# front; under numpy >= 2 / NEP 50 the same source would accumulate in float32).  Array-array
# promotion is the same in both: a terminated path's b1 = append(b, 0.0) is float64 (so its
# deltas are float64), a non-terminated path's b1 = append(b, b[-1]) stays float32 and so do
# its deltas (float32 rewards + float32(gamma) * b1[1:] - b1[:-1]).
# --------------------------------------------------------------------------------------


def init_mlp_baseline(inp_dim: int, hidden=(128, 128), seed: int | None = None):
    """MLPBaseline.model layers (mlp_baseline.py:20-27): Linear(n+4 -> h1) ReLU ... Linear(-> 1),
    default torch init in layer order."""
    if seed is not None:
        torch.manual_seed(seed)
    sizes = (inp_dim + 4,) + tuple(hidden) + (1,)
    layers = [nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)]
    return [(l.weight.data.clone(), l.bias.data.clone()) for l in layers]


def mlp_baseline_features(paths) -> np.ndarray:
    """MLPBaseline._features (mlp_baseline.py:36-59) for inp='obs', as float32 (:100).  A path
    may carry 't0' (engine lanes: a trajectory begun in an earlier rollout); mjrl paths
    always start at 0."""
    o = np.concatenate([p["observations"] for p in paths])
    o = np.clip(o, -10, 10) / 10.0
    N_, n = o.shape
    feat = np.ones((N_, n + 4))
    feat[:, :n] = o
    k = 0
    for p in paths:
        l = len(p["rewards"])
        al = (np.arange(l) + p.get("t0", 0)) / 1000.0
        for j in range(4):
            feat[k:k + l, -4 + j] = al ** (j + 1)
        k += l
    return feat.astype("float32")


def mlp_baseline_predict(layers, feat: np.ndarray) -> np.ndarray:
    """model(feat) (mlp_baseline.py:99-108): Linear/ReLU chain in fp32."""
    x = torch.from_numpy(feat)
    for i, (W, b) in enumerate(layers):
        x = F.linear(x, W, b)
        if i < len(layers) - 1:
            x = torch.relu(x)
    return x.detach().numpy().ravel()


def discount_sum(x, gamma: float, terminal: float = 0.0) -> np.ndarray:
    """process_samples.py:37-45 with numpy-1.21 scalar promotion (float64 accumulation)."""
    x = np.asarray(x, dtype=np.float64)
    y = []
    run_sum = terminal
    for t in range(len(x) - 1, -1, -1):
        run_sum = x[t] + gamma * run_sum
        y.append(run_sum)
    return np.array(y[::-1])


def compute_returns(paths, gamma: float) -> None:
    """process_samples.py:3-5."""
    for p in paths:
        p["returns"] = discount_sum(p["rewards"], gamma)


def compute_advantages(paths, predict, gamma: float, gae_lambda=None, normalize: bool = False) -> None:
    """process_samples.py:7-35; `predict(path)` returns the path's baseline (float32)."""
    if gae_lambda is None or gae_lambda < 0.0 or gae_lambda > 1.0:
        for p in paths:
            p["baseline"] = predict(p)
            p["advantages"] = p["returns"] - p["baseline"]
        if normalize:
            alladv = np.concatenate([p["advantages"] for p in paths])
            mean_adv, std_adv = alladv.mean(), alladv.std()
            for p in paths:
                p["advantages"] = (p["advantages"] - mean_adv) / (std_adv + 1e-8)
    else:
        for p in paths:
            b = p["baseline"] = predict(p)
            b1 = np.append(b, 0.0 if p["terminated"] else b[-1])
            td = p["rewards"] + gamma * b1[1:] - b1[:-1]
            p["advantages"] = discount_sum(td, gamma * gae_lambda)
        if normalize:
            alladv = np.concatenate([p["advantages"] for p in paths])
            mean_adv, std_adv = alladv.mean(), alladv.std()
            for p in paths:
                p["advantages"] = (p["advantages"] - mean_adv) / (std_adv + 1e-8)


def whiten_advantages(paths, eps: float = 1e-6):
    """BatchREINFORCE.process_paths advantage whitening + return stats
    (batch_reinforce.py:280-293)."""
    adv = np.concatenate([p["advantages"] for p in paths])
    adv = (adv - np.mean(adv)) / (np.std(adv) + eps)
    # sum() of float32 scalars accumulates in float64 under numpy 1.21 (scalar promotion)
    path_returns = [sum(np.asarray(p["rewards"], dtype=np.float64)) for p in paths]
    return adv, [np.mean(path_returns), np.std(path_returns), np.amin(path_returns), np.amax(path_returns)]


def lanes_to_paths(done: np.ndarray, rewards: np.ndarray, obs: np.ndarray, steps0: np.ndarray):
    """Split rollout-engine lane buffers [T, B] into mjrl-style paths (test helper): a lane's
    trajectory ends at a done flag (terminated) or at the end of the buffer (not
    terminated).  Returns (paths, rows) with rows[i] = the (t, b) pairs of path i."""
    T, B = done.shape
    paths, rows = [], []
    for b in range(B):
        start = 0
        for t in range(T):
            if done[t, b] or t == T - 1:
                ts = np.arange(start, t + 1)
                paths.append(dict(observations=obs[ts, b], rewards=rewards[ts, b], terminated=bool(done[t, b]),
                                  t0=int(steps0[b]) if start == 0 else 0))
                rows.append((ts, b))
                start = t + 1
    return paths, rows


# --------------------------------------------------------------------------------------
# NPG policy update — mjrl/mjrl/algos/npg_cg.py:60-199 (CPI_surrogate, HVP, train_from_paths),
# mjrl/mjrl/algos/batch_reinforce.py:58-62 (flat_vpg), mjrl/mjrl/policies/gaussian_mlp.py
# (mean_LL :110-126, likelihood_ratio :138-142, mean_kl :144-155, set_param_values :71-94),
# mjrl/mjrl/utils/cg_solve.py:3-23.  torch-CPU float32 autograd, as the reference.
# --------------------------------------------------------------------------------------


def policy_param_shapes(S: int, A: int, hidden=(32, 32)):
    """Shapes of MLP.trainable_params in order: fc weights/biases then log_std."""
    sizes = (S,) + tuple(hidden) + (A,)
    shapes = []
    for i in range(len(sizes) - 1):
        shapes += [(sizes[i + 1], sizes[i]), (sizes[i + 1],)]
    return shapes + [(A,)]


def _unflatten(flat, shapes, grad=False):
    out, i = [], 0
    for sh in shapes:
        n = int(np.prod(sh))
        t = torch.from_numpy(np.asarray(flat[i:i + n], dtype=np.float32).reshape(sh).copy())
        out.append(t.requires_grad_(grad))
        i += n
    return out


def _policy_mean_ll(params, obs_t, act_t, A):
    """MLP.mean_LL (gaussian_mlp.py:110-126) through FCNetwork.forward (fc_network.py:45-55,
    default in_shift/in_scale: (x - 0) / (1 + 1e-8) == x in float32)."""
    out = obs_t
    layers = params[:-1]
    n_lin = len(layers) // 2
    for j in range(n_lin):
        out = F.linear(out, layers[2 * j], layers[2 * j + 1])
        if j < n_lin - 1:
            out = torch.tanh(out)
    log_std = params[-1]
    zs = (act_t - out) / torch.exp(log_std)
    LL = -0.5 * torch.sum(zs ** 2, dim=1) + -torch.sum(log_std) + -0.5 * A * np.log(2 * np.pi)
    return out, LL


def _mean_kl(new_mean, new_ls, old_mean, old_ls):
    old_std, new_std = torch.exp(old_ls), torch.exp(new_ls)
    Nr = (old_mean - new_mean) ** 2 + old_std ** 2 - new_std ** 2
    Dr = 2 * new_std ** 2 + 1e-8
    return torch.mean(torch.sum(Nr / Dr + new_ls - old_ls, dim=1))


def npg_hvp(flat, shapes, obs, act, v, damping=1e-4):
    """NPG.HVP (npg_cg.py:87-106): d/dtheta <grad mean_kl(new || old), v> + damping * v at
    new == old, hvp_sample_frac = 1."""
    A = shapes[-1][0]
    obs_t, act_t = torch.from_numpy(np.asarray(obs)).float(), torch.from_numpy(np.asarray(act)).float()
    new = _unflatten(flat, shapes, grad=True)
    old = _unflatten(flat, shapes)
    old_mean, _ = _policy_mean_ll(old, obs_t, act_t, A)
    new_mean, _ = _policy_mean_ll(new, obs_t, act_t, A)
    kl = _mean_kl(new_mean, new[-1], old_mean, old[-1])
    g = torch.autograd.grad(kl, new, create_graph=True)
    flat_g = torch.cat([x.contiguous().view(-1) for x in g])
    h = torch.sum(flat_g * torch.from_numpy(np.asarray(v, dtype=np.float32)))
    hv = torch.autograd.grad(h, new)
    return np.concatenate([x.contiguous().view(-1).data.numpy() for x in hv]) + damping * np.asarray(v, np.float32)


def _cpi_surrogate(new_flat, old_flat, shapes, obs, act, adv):
    A = shapes[-1][0]
    obs_t, act_t = torch.from_numpy(np.asarray(obs)).float(), torch.from_numpy(np.asarray(act)).float()
    new = _unflatten(new_flat, shapes, grad=True)
    old = _unflatten(old_flat, shapes)
    _, LL_old = _policy_mean_ll(old, obs_t, act_t, A)
    _, LL_new = _policy_mean_ll(new, obs_t, act_t, A)
    LR = torch.exp(LL_new - LL_old)
    return torch.mean(LR * torch.from_numpy(np.asarray(adv)).float()), new


def npg_vpg(flat, shapes, obs, act, adv_w):
    """BatchREINFORCE.flat_vpg (batch_reinforce.py:58-62) at new == old."""
    surr, new = _cpi_surrogate(flat, flat, shapes, obs, act, adv_w)
    g = torch.autograd.grad(surr, new)
    return np.concatenate([x.contiguous().view(-1).data.numpy() for x in g]), float(surr.data.numpy())


def cg_solve(f_Ax, b, cg_iters=10, residual_tol=1e-10):
    """mjrl/mjrl/utils/cg_solve.py:3-23 (x_0 ignored: starts from zeros)."""
    x = np.zeros_like(b)
    r = b.copy()
    p = r.copy()
    rdotr = r.dot(r)
    for _ in range(cg_iters):
        z = f_Ax(p)
        v = rdotr / p.dot(z)
        x += v * p
        r -= v * z
        newrdotr = r.dot(r)
        mu = newrdotr / rdotr
        p = r + mu * p
        rdotr = newrdotr
        if rdotr < residual_tol:
            break
    return x


def npg_update(flat, shapes, obs, act, adv, step=0.1, damping=1e-4, cg_iters=10, min_log_std=-2.0):
    """NPG.train_from_paths (npg_cg.py:113-199) without logging: whitening
    (batch_reinforce.py:284-285), VPG, CG on the HVP, alpha = sqrt(|step / (g.npg + 1e-20)|),
    params += alpha * npg with the log_std clamp, surr_after."""
    adv = np.asarray(adv, dtype=np.float64)
    adv_w = (adv - np.mean(adv)) / (np.std(adv) + 1e-6)
    flat = np.asarray(flat, dtype=np.float32)
    vpg, surr_before = npg_vpg(flat, shapes, obs, act, adv_w)
    npg = cg_solve(lambda v: npg_hvp(flat, shapes, obs, act, v, damping), vpg, cg_iters=cg_iters)
    alpha = np.sqrt(np.abs(step / (np.dot(vpg.T, npg) + 1e-20)))
    new = flat + alpha * npg
    new32 = np.asarray(new).astype(np.float32)
    A = shapes[-1][0]
    new32[-A:] = np.maximum(new32[-A:], np.float32(min_log_std))  # torch.clamp(log_std, min_log_std)
    surr_after, _ = _cpi_surrogate(new32, flat, shapes, obs, act, adv_w)
    return dict(adv_whitened=adv_w, vpg=vpg, npg=npg, alpha=float(alpha), params1=new32,
                surr_before=surr_before, surr_after=float(surr_after.data.numpy()))
