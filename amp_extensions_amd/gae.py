"""Returns, the MLP value baseline and GAE on the device: the consumer of the sampler's
output in the reference's policy step (mjrl BatchREINFORCE.train_step,
mjrl/mjrl/algos/batch_reinforce.py:176-180, and process_paths :271-297).

Two layouts share the same kernels (include/amx_hip.h, "segment grid"):
  * the rollout engine's lane buffers ([T, B] rows, several trajectories per lane separated
    by done flags, trajectories that run past the buffer bootstrapped as non-terminated);
  * concatenated mjrl path dicts (`process_samples`), one lane per path — a drop-in for
    `process_samples.compute_returns` + `compute_advantages` (mjrl/mjrl/utils/process_samples.py).
The value MLP is the reference's MLPBaseline (mjrl/mjrl/baselines/mlp_baseline.py:10-108):
features [clip(obs,-10,10)/10, (t/1000)^1..4] -> Linear/ReLU ... -> Linear(., 1), run on the
MFMA GEMM with the hidden widths zero-padded to 128.  Fitting the baseline (Adam) belongs to
the learner and stays with the caller's torch model; call `sync_from` after each fit.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from .engine import AmxContext, round_up


def init_mlp_baseline_params(inp_dim: int, hidden=(128, 128), seed: int | None = None):
    """Layers of MLPBaseline.model (mlp_baseline.py:20-27): nn.Linear(n+4 -> h1), ReLU, ...,
    nn.Linear(-> 1), default torch init drawn in layer order (after torch.manual_seed(seed)
    when a seed is given)."""
    if seed is not None:
        torch.manual_seed(seed)
    sizes = (inp_dim + 4,) + tuple(hidden) + (1,)
    layers = [nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)]
    return [(l.weight.data.clone(), l.bias.data.clone()) for l in layers]


class DeviceMLPBaseline:
    """MLPBaseline.predict on the device.  Workspace rows: [feat kf | h0 | h1 | ...] with
    kf = round_up(S+4, 32) and every hidden width padded to a multiple of 128."""

    def __init__(self, ctx: AmxContext, layers):
        self.ctx = ctx
        self.kf = round_up(ctx.S + 4, 32)
        self._ws = None
        self.sync_from(layers)

    @classmethod
    def from_mjrl(cls, ctx: AmxContext, baseline):
        """Build from an mjrl `MLPBaseline` (its nn.Sequential of Linear/ReLU)."""
        return cls(ctx, cls._layers_of(baseline))

    @staticmethod
    def _layers_of(baseline):
        return [(m.weight.data, m.bias.data) for m in baseline.model if isinstance(m, nn.Linear)]

    def sync_from(self, layers) -> None:
        """Upload (W [out, in], b) per layer; accepts the list or an mjrl MLPBaseline."""
        if hasattr(layers, "model"):
            layers = self._layers_of(layers)
        c, dev = self.ctx, self.ctx.device
        if len(layers) < 2:
            raise ValueError("MLPBaseline needs at least one hidden layer")
        if layers[0][0].shape[1] != c.S + 4 or layers[-1][0].shape[0] != 1:
            raise ValueError(f"baseline layers must map {c.S + 4} features to 1 value")
        widths = [int(W.shape[0]) for W, _ in layers[:-1]]
        self.Hp = [round_up(h, 128) for h in widths]
        self.col = [0, self.kf]
        for hp in self.Hp:
            self.col.append(self.col[-1] + hp)
        self.ldv = self.col[-1]
        self.W, self.b = [], []
        k_in, kin_pad = c.S + 4, self.kf
        for i, (W, b) in enumerate(layers[:-1]):
            Wp = torch.zeros(self.Hp[i], kin_pad, dtype=torch.float32)
            Wp[: W.shape[0], :k_in] = torch.as_tensor(W).float()
            bp = torch.zeros(self.Hp[i], dtype=torch.float32)
            bp[: W.shape[0]] = torch.as_tensor(b).float()
            self.W.append(Wp.to(dev).contiguous())
            self.b.append(bp.to(dev).contiguous())
            k_in, kin_pad = W.shape[0], self.Hp[i]
        W, b = layers[-1]
        wh = torch.zeros(self.Hp[-1], dtype=torch.float32)
        wh[: W.shape[1]] = torch.as_tensor(W).float().reshape(-1)
        self.w_head = wh.to(dev).contiguous()
        self.b_head = torch.as_tensor(b).float().reshape(1).to(dev).contiguous()

    def workspace(self, rows: int) -> torch.Tensor:
        rp = max(round_up(rows, 128), 128)
        if self._ws is None or self._ws.shape[0] < rp or self._ws.shape[1] != self.ldv:
            self._ws = torch.zeros(rp, self.ldv, dtype=torch.float32, device=self.ctx.device)
            self._v = torch.zeros(rp, dtype=torch.float32, device=self.ctx.device)
        return self._ws

    def predict_grid(self, rows: int, T: int, L: int, obs: torch.Tensor, ldo: int, end: torch.Tensor, stride: int,
                     lengths: torch.Tensor | None = None, t0: torch.Tensor | None = None,
                     base: torch.Tensor | None = None) -> torch.Tensor:
        """Baseline values of every grid row (rows = row-space size) -> f32 [rows_pad]."""
        c = self.ctx
        ws = self.workspace(rows)
        rp = round_up(rows, 128)
        N.check(c.lib.amx_value_features(c.h, T, L, _ptr(lengths), _ptr(t0), _ptr(base), stride, end.data_ptr(),
                                         obs.data_ptr(), ldo, ws.data_ptr(), self.ldv, c.stream), "amx_value_features")
        for i in range(len(self.Hp)):
            K = self.kf if i == 0 else self.Hp[i - 1]
            A = ws[:, self.col[i]:]
            N.check(c.lib.amx_gemm_bias_act(c.h, 1, rp, self.Hp[i], K, A.data_ptr(), self.ldv, 0, self.W[i].data_ptr(),
                                            K, 0, self.b[i].data_ptr(), 0, ws.data_ptr(), self.ldv, 0, self.col[i + 1],
                                            1, c.stream), "amx_gemm_bias_act")
        h = ws[:, self.col[-2]:]
        N.check(c.lib.amx_value_head(c.h, rp, h.data_ptr(), self.ldv, self.Hp[-1], self.w_head.data_ptr(),
                                     self.b_head.data_ptr(), self._v.data_ptr(), c.stream), "amx_value_head")
        return self._v[:rp]


def _ptr(t):
    return None if t is None else t.data_ptr()


def gamma_lambda(gamma: float, gae_lambda) -> float:
    """compute_advantages' mode switch (process_samples.py:10): GAE for 0 <= lambda <= 1,
    the standard returns - baseline mode otherwise (encoded as a negative value)."""
    if gae_lambda is None or gae_lambda < 0.0 or gae_lambda > 1.0:
        return -1.0
    return float(gamma) * float(gae_lambda)


def gae_grid(ctx: AmxContext, T: int, L: int, end, rew, rstride: int, v, gamma: float, gae_lambda, stride: int,
             ret: torch.Tensor, adv: torch.Tensor, lengths=None, base=None, rbase=None) -> None:
    N.check(ctx.lib.amx_gae(ctx.h, T, L, _ptr(lengths), _ptr(base), stride, end.data_ptr(), rew.data_ptr(),
                            _ptr(rbase), rstride, v.data_ptr(), float(gamma), gamma_lambda(gamma, gae_lambda),
                            ret.data_ptr(), adv.data_ptr(), ctx.stream), "amx_gae")


def whiten_grid(ctx: AmxContext, T: int, L: int, adv: torch.Tensor, stride: int, eps: float = 1e-6,
                out: torch.Tensor | None = None, lengths=None, base=None) -> tuple[torch.Tensor, torch.Tensor]:
    """(adv - mean) / (std + eps) over the grid rows (batch_reinforce.py:284-285); returns
    (out, stats[mean, std]) as device tensors."""
    out = adv if out is None else out
    stats = torch.empty(2, dtype=torch.float64, device=adv.device)
    N.check(ctx.lib.amx_adv_whiten(ctx.h, T, L, _ptr(lengths), _ptr(base), stride, adv.data_ptr(), float(eps),
                                   out.data_ptr(), stats.data_ptr(), ctx.stream), "amx_adv_whiten")
    return out, stats


def process_samples(paths, baseline: DeviceMLPBaseline, gamma: float, gae_lambda=None, normalize: bool = False):
    """mjrl `compute_returns(paths, gamma)` + `compute_advantages(paths, baseline, gamma,
    gae_lambda, normalize)` (process_samples.py:3-35) on the device for a list of path dicts.
    Writes path['returns'] (f64), path['baseline'] (f32) and path['advantages'] (f64) like
    the reference; returns the device tensors (concatenated path order)."""
    c = baseline.ctx
    dev = c.device
    lens = np.array([len(p["rewards"]) for p in paths], dtype=np.int64)
    n_rows = int(lens.sum())
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    obs = torch.from_numpy(np.ascontiguousarray(np.concatenate([p["observations"] for p in paths]),
                                                dtype=np.float64)).to(dev)
    rew = torch.from_numpy(np.concatenate([np.asarray(p["rewards"], dtype=np.float32) for p in paths])).to(dev)
    end = np.zeros(n_rows, dtype=np.uint8)
    for p, o, l in zip(paths, offs, lens):
        if l:
            end[o + l - 1] = 1 if p.get("terminated", True) else 2
    end_d = torch.from_numpy(end).to(dev)
    lens_d = torch.from_numpy(lens.astype(np.int32)).to(dev)
    base_d = torch.from_numpy(offs).to(dev)
    T, L = int(lens.max(initial=0)), len(paths)
    v = baseline.predict_grid(n_rows, T, L, obs, c.S, end_d, 1, lengths=lens_d, base=base_d)
    ret = torch.empty(max(n_rows, 1), dtype=torch.float64, device=dev)
    adv = torch.empty_like(ret)
    gae_grid(c, T, L, end_d, rew, 1, v, gamma, gae_lambda, 1, ret, adv, lengths=lens_d, base=base_d, rbase=base_d)
    if normalize:  # process_samples.py:23-28 / 30-35 (eps 1e-8)
        whiten_grid(c, T, L, adv, 1, eps=1e-8, lengths=lens_d, base=base_d)
    ret_h, adv_h, v_h = ret.cpu().numpy(), adv.cpu().numpy(), v[:n_rows].cpu().numpy()
    for p, o, l in zip(paths, offs, lens):
        p["returns"] = ret_h[o:o + l].copy()
        p["baseline"] = v_h[o:o + l].copy()
        p["advantages"] = adv_h[o:o + l].copy()
    return ret[:n_rows], adv[:n_rows], v[:n_rows]
