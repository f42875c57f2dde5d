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

from .costs import GAILCost, RBFLinearCost, cost_input, device_discrepancy
from .dist import feature_mean


def _device_rows(paths, key: str, dev):
    """The paths' `key` rows as the device tensor sample_points already holds (sampler._last_rows)
    when the paths' arrays are consecutive views of its read-only host copy; else None."""
    from .sampler import _last_rows
    ent = _last_rows.get(key)
    if ent is None or ent[1].device != dev:
        return None
    base, rows = ent
    if base.flags.writeable:
        return None
    arrs = [p[key] for p in paths]
    if not arrs or any(a.base is not base for a in arrs):
        return None
    row = base.strides[0]
    start = arrs[0].__array_interface__["data"][0]
    off = start
    for a in arrs:
        if a.__array_interface__["data"][0] != off or a.shape[1:] != base.shape[1:] or a.flags.writeable:
            return None
        off += a.shape[0] * row
    r0 = (start - base.__array_interface__["data"][0]) // row
    return rows[r0:r0 + (off - start) // row]


def _rows(paths, key: str) -> np.ndarray:
    """np.concatenate([p[key] for p in paths]) -- without the copy when the paths' arrays are
    consecutive views of one buffer (sample_points returns them so)."""
    arrs = [p[key] for p in paths]
    a0 = arrs[0]
    base = a0.base
    if base is not None and all(a.base is base and a.flags.c_contiguous and a.dtype == a0.dtype for a in arrs):
        row = a0.strides[0]
        start = a0.__array_interface__["data"][0]
        off = start
        for a in arrs:
            if a.__array_interface__["data"][0] != off or a.shape[1:] != a0.shape[1:]:
                break
            off += a.shape[0] * row
        else:
            n = sum(a.shape[0] for a in arrs)
            return np.lib.stride_tricks.as_strided(a0, shape=(n,) + a0.shape[1:], strides=a0.strides)
    return np.concatenate(arrs)


_copy_streams: dict = {}


def _upload(paths, dev):
    """The paths' float64 rows on the device as float32 (the reference's .float() of its
    tensors), copied on a side stream: actions and observations first (the disagreement's
    inputs), then the next states, which `next_rows()` hands to the current stream when the
    caller needs them.  The sampler's paths are views of one pinned buffer, so the copies are
    asynchronous DMA; other arrays are copied synchronously by torch.  Paths that are views of
    the last sample_points call's read-only host arrays are read from its device rows instead."""
    main = torch.cuda.current_stream(dev)
    d = [_device_rows(paths, k, dev) for k in ("observations", "actions", "next_observations")]
    if all(x is not None for x in d):  # sample_points' own device rows: no upload
        return d[0].float(), d[1].float(), lambda: d[2].float()
    cs = _copy_streams.get(dev)
    if cs is None:
        cs = _copy_streams[dev] = torch.cuda.Stream(dev)
    cs.wait_stream(main)
    with torch.cuda.stream(cs):
        a64 = torch.from_numpy(_rows(paths, "actions")).to(dev, non_blocking=True)
        o64 = torch.from_numpy(_rows(paths, "observations")).to(dev, non_blocking=True)
        e_sa = torch.cuda.Event()
        e_sa.record(cs)
        n64 = torch.from_numpy(_rows(paths, "next_observations")).to(dev, non_blocking=True)
        e_n = torch.cuda.Event()
        e_n.record(cs)
    main.wait_event(e_sa)
    for t in (a64, o64, n64):
        t.record_stream(main)  # (allocated on the copy stream, consumed on this one)

    def next_rows():
        main.wait_event(e_n)
        return n64.float()
    return o64.float(), a64.float(), next_rows


def relabel_paths(paths, reward_func, ensemble, cost_input_type: str = "ss", allreduce=None) -> dict:
    """`cost_input_type` builds the fit_cost input ('ss' or 'sa', batch_reinforce.py:107-110);
    the per-sample rewards use reward_func's own input_type (get_bonus_costs).  With
    `ensemble` None the GAIL path replaces the rewards with -get_costs([s, s'])
    (batch_reinforce.py:146-158)."""
    infos = {"int": [], "ext": [], "reward": [], "ep_len": []}
    if cost_input_type not in ("ss", "sa"):
        # the reference leaves cost_input unbound for any other value
        raise NotImplementedError(f"cost_input_type {cost_input_type!r}: batch_reinforce builds only 'ss' / 'sa'")
    dev = reward_func.ctx.device
    lens = [len(p["observations"]) for p in paths]
    obs, act, next_rows = _upload(paths, dev)
    bonus_v = ipm_v = None
    if isinstance(reward_func, RBFLinearCost):
        if ensemble is None:
            raise ValueError("the MMD relabel needs the ensemble (batch_reinforce.py:147 asserts a GAIL cost)")
        # the disagreement first: its ensemble forward runs while the next states upload
        disc = device_discrepancy(ensemble, obs, act)
        nxt = next_rows()
        x_fit = cost_input(cost_input_type, obs, act, nxt)
        phi_fit, tot = reward_func.map.embed(x_fit)
        mean = feature_mean(tot, float(x_fit.shape[0]), allreduce if allreduce is not None else (lambda t: t))
        infos["mb_mmd"] = reward_func.fit_w(mean.contiguous(), 1.0)           # batch_reinforce.py:113
        if reward_func.input_type == cost_input_type:
            phi = phi_fit
        else:
            phi = reward_func.get_rep(cost_input(reward_func.input_type, obs, act, nxt, reward_func.motion))
        reward, ipm, wb = reward_func._values(phi, disc, ensemble.threshold)
        bonus_v, ipm_v = wb.cpu().numpy(), ipm.cpu().numpy()
    elif isinstance(reward_func, GAILCost):
        nxt = next_rows()
        # the reference scores [s, s'] here (:152-165); an AMP-feature discriminator scores AMP(s, s')
        x_ss = (cost_input("amp", obs, act, nxt, reward_func.motion) if reward_func.input_type == "amp"
                else torch.cat([obs, nxt], dim=-1))
        if ensemble is not None:
            cost, ci = reward_func.get_bonus_costs(obs, act, ensemble, next_states=nxt)
            reward = -cost.view(-1)
            bonus_v, ipm_v = ci["bonus"].view(-1).cpu().numpy(), ci["ipm"].view(-1).cpu().numpy()
        else:
            reward = -reward_func.get_costs(x_ss).view(-1)                             # :152-158
    else:
        raise TypeError("reward_func must be an RBFLinearCost or GAILCost")
    rew = reward.cpu().numpy()
    if bonus_v is not None and lens:
        # the per-path sums of batch_reinforce.py:135-136 for all paths in one pass (float32
        # segment sums: np.sum's pairwise order differs in the last bits, inside the values' own
        # fp32 tolerance)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        isums = -np.add.reduceat(bonus_v, starts)
        esums = -np.add.reduceat(ipm_v, starts)
        infos["int"] = list(isums)
        infos["ext"] = list(esums)
        infos["reward"] = list(esums + isums)
        infos["ep_len"] = list(lens)
    o = 0
    for p, T in zip(paths, lens):
        p["rewards"] = rew[o:o + T].copy()  # :144 (reward = -cost)
        o += T
    if isinstance(reward_func, GAILCost):
        infos["on_policy_gail_cost"] = reward_func.get_costs(x_ss)                     # :160-165
    else:
        infos["bonus_mmd"] = np.concatenate([-1.0 * p["rewards"] for p in paths]).mean() - \
            float(reward_func.get_expert_cost())                                 # :169
    return infos
