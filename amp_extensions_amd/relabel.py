"""Reward relabel of collected paths — the block of BatchREINFORCE.train_step that calls the
hot path (mjrl/mjrl/algos/batch_reinforce.py:103-169), on the device cost objects.

One device pass over all samples replaces the reference's per-trajectory Python loop
(the per-path numbers are sliced out afterwards), and the ensemble disagreement is taken
from the same device ensemble.  `allreduce` (optional) sums a device tensor across ranks
for the global feature mean of fit_cost when the rollout is sharded.
"""
from __future__ import annotations

import numpy as np
import torch

from .costs import GAILCost, RBFLinearCost
from .dist import feature_mean


def relabel_paths(paths, reward_func, ensemble, cost_input_type: str = "ss", allreduce=None) -> dict:
    infos = {"int": [], "ext": [], "reward": [], "ep_len": []}
    if cost_input_type != "ss":
        raise NotImplementedError("the humanoid MILO path uses the 'ss' cost input")
    dev = reward_func.ctx.device
    lens = [len(p["observations"]) for p in paths]
    obs = torch.from_numpy(np.concatenate([p["observations"] for p in paths])).float().to(dev)
    nxt = torch.from_numpy(np.concatenate([p["next_observations"] for p in paths])).float().to(dev)
    act = torch.from_numpy(np.concatenate([p["actions"] for p in paths])).float().to(dev)
    if isinstance(reward_func, RBFLinearCost):
        x = torch.cat([obs, nxt], dim=1)
        phi, tot = reward_func.map.embed(x)
        mean = feature_mean(tot, float(x.shape[0]), allreduce if allreduce is not None else (lambda t: t))
        infos["mb_mmd"] = reward_func.fit_w(mean.contiguous(), 1.0)           # batch_reinforce.py:113
        disc = ensemble.get_action_discrepancy(obs, act)
        reward, ipm, wb = reward_func._values(phi, disc, ensemble.threshold)
        bonus_v, ipm_v = wb.cpu().numpy(), ipm.cpu().numpy()
    elif isinstance(reward_func, GAILCost):
        cost, ci = reward_func.get_bonus_costs(obs, act, ensemble, next_states=nxt)
        reward = -cost.view(-1)
        bonus_v, ipm_v = ci["bonus"].view(-1).cpu().numpy(), ci["ipm"].view(-1).cpu().numpy()
    else:
        raise TypeError("reward_func must be an RBFLinearCost or GAILCost")
    rew = reward.cpu().numpy()
    o = 0
    for p, T in zip(paths, lens):
        isum = -np.sum(bonus_v[o:o + T])    # batch_reinforce.py:135
        esum = -np.sum(ipm_v[o:o + T])      # :136
        infos["int"].append(isum)
        infos["ext"].append(esum)
        infos["reward"].append(esum + isum)
        infos["ep_len"].append(T)
        p["rewards"] = rew[o:o + T].copy()  # :144 (reward = -cost)
        o += T
    if isinstance(reward_func, RBFLinearCost):
        infos["bonus_mmd"] = np.concatenate([-1.0 * p["rewards"] for p in paths]).mean() - \
            float(reward_func.get_expert_cost())                                 # :169
    return infos
