"""Device copy of the mjrl Gaussian MLP policy (mjrl/mjrl/policies/gaussian_mlp.py:7-104).

Only the sampling surface the rollout needs (get_action on B lanes at once) runs on the
GPU; the learner (NPG/TRPO) is out of scope and keeps the host-side policy object.  Call
`sync_from(params)` after every policy update to refresh the device weights.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from .engine import AmxContext


def init_mlp_policy_params(S: int, A: int, hidden=(32, 32), seed=100, init_log_std=-0.25):
    """Parameters exactly as mjrl MLP.__init__ draws them (gaussian_mlp.py:28-40): seeded,
    FCNetwork layers in order, last layer weight and bias scaled by 1e-2."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    sizes = (S,) + tuple(hidden) + (A,)
    layers = [nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)]
    layers[-1].weight.data = 1e-2 * layers[-1].weight.data
    layers[-1].bias.data = 1e-2 * layers[-1].bias.data
    return [(l.weight.data.clone(), l.bias.data.clone()) for l in layers], torch.ones(A) * init_log_std


class DevicePolicy:
    """Tanh MLP(S -> H1 -> H2 -> A) + exp(log_std) Gaussian noise, on the device."""

    def __init__(self, ctx: AmxContext, layers, log_std, seed: int = 0):
        if len(layers) != 3:
            raise NotImplementedError("the device policy kernel supports two hidden layers (mjrl default)")
        self.ctx = ctx
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.sync_from(layers, log_std)

    @classmethod
    def from_mjrl(cls, ctx: AmxContext, policy, seed: int = 0):
        """Build from an mjrl `MLP` object: model.fc_layers for the mean, and log_std_val -- the
        float64 copy mjrl's get_action draws its noise with and reports as agent_infos['log_std']
        (gaussian_mlp.py:53, 95-104), refreshed only by set_param_values -- for the noise."""
        layers = [(l.weight.data, l.bias.data) for l in policy.model.fc_layers]
        return cls(ctx, layers, np.asarray(policy.log_std_val, np.float64), seed)

    def sync_from(self, layers, log_std) -> None:
        dev = self.ctx.device
        self.W = [torch.as_tensor(W).float().to(dev).contiguous() for (W, _) in layers]
        self.b = [torch.as_tensor(b).float().to(dev).contiguous() for (_, b) in layers]
        self.H1, self.H2 = self.W[0].shape[0], self.W[1].shape[0]
        assert self.W[0].shape[1] == self.ctx.S and self.W[2].shape[0] == self.ctx.A
        # log_std_val = float64(log_std); noise scale = np.exp(log_std_val) (gaussian_mlp.py:53,102)
        ls = np.float64(torch.as_tensor(log_std).detach().cpu().numpy().ravel())
        self.log_std_val = ls
        scale = torch.from_numpy(np.exp(ls)).to(dev)
        c = self.ctx
        n = int(c.lib.amx_policy_blob_floats(c.h, self.H1, self.H2))
        if n <= 0:
            raise ValueError("amx_policy_blob_floats failed")
        # a re-sync of the same shapes rewrites the device buffers in place: HIP graphs captured
        # around this policy (sample_points' chunk graphs) keep reading the current parameters
        if getattr(self, "blob", None) is not None and self.blob.numel() == n and self.noise_scale.shape == scale.shape:
            self.noise_scale.copy_(scale)
        else:
            self.noise_scale = scale
            self.blob = torch.zeros(n, dtype=torch.float32, device=dev)  # (the tail past the image: LDS-DMA padding)
        N.check(c.lib.amx_policy_pack(c.h, self.W[0].data_ptr(), self.b[0].data_ptr(), self.H1, self.W[1].data_ptr(),
                                      self.b[1].data_ptr(), self.H2, self.W[2].data_ptr(), self.b[2].data_ptr(),
                                      self.blob.data_ptr(), c.stream), "amx_policy_pack")

    def act(self, ob: torch.Tensor, B: int, out: torch.Tensor, counter: int, noise: torch.Tensor | None = None,
            eval_mode: bool = False, mean_out: torch.Tensor | None = None, x0: torch.Tensor | None = None,
            counter_dev: torch.Tensor | None = None, row_exp: torch.Tensor | None = None,
            shared_x0: bool = False) -> torch.Tensor:
        """Actions of B lanes into `out` [B, A] f64.  `x0` (the ensemble workspace's activation
        buffer [M, B_pad, ldk]) fuses the ensemble's input assembly into the same launch
        (`shared_x0`: once, into model 0's rows, for the f16x3 GEMMs' k_shared slice);
        `row_exp` (the workspace's [M, L+1, B_pad] f16x3 exponent slots) also writes slot 0 and
        resets the others, as amx_assemble_input_rexp.  `counter_dev` (int64 [1] on the device):
        the Philox counter is counter_dev[0] + `counter` (amx_policy_act_dev: HIP-graph replays
        draw fresh noise)."""
        c = self.ctx
        x0p = None if x0 is None else x0.data_ptr()
        sm = 0 if (x0 is None or shared_x0) else x0.stride(0)
        ldk = 0 if x0 is None else x0.stride(1)
        rx = (None, 0, 0, 0) if row_exp is None else (row_exp.data_ptr(), row_exp.stride(0), row_exp.stride(1),
                                                      row_exp.shape[1])
        if counter_dev is not None:
            N.check(c.lib.amx_policy_act_dev(
                c.h, ob.data_ptr(), B, self.blob.data_ptr(), self.H1, self.H2, self.noise_scale.data_ptr(),
                None if noise is None else noise.data_ptr(), self.seed, counter_dev.data_ptr(),
                int(counter) & 0xFFFFFFFFFFFFFFFF, int(eval_mode),
                out.data_ptr(), None if mean_out is None else mean_out.data_ptr(), x0p, sm, ldk, *rx, c.stream),
                "amx_policy_act_dev")
            return out
        N.check(c.lib.amx_policy_act(
            c.h, ob.data_ptr(), B, self.blob.data_ptr(), self.H1, self.H2, self.noise_scale.data_ptr(),
            None if noise is None else noise.data_ptr(), self.seed, int(counter) & 0xFFFFFFFFFFFFFFFF,
            int(eval_mode), out.data_ptr(), None if mean_out is None else mean_out.data_ptr(), x0p, sm, ldk, *rx,
            c.stream), "amx_policy_act")
        return out
