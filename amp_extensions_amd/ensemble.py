"""Drop-in `DynamicsEnsemble` surface (milo/milo/dynamics.py:19-165) over the device ensemble.

Inference only: ensemble training (DynamicsModel.train*, dynamics.py:236-378) is out of
scope.  Weights come from the reference's own checkpoint format (`save_ensemble`: a list of
{'model': BasicMLP state_dict, 'optim': ...}, dynamics.py:110-131), loaded with
torch.load(weights_only=True), or from a seeded random init that draws exactly what
DynamicsModel.__init__ draws.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .engine import AmxContext, DeviceEnsemble


def basic_mlp_layer_shapes(S: int, A: int, hidden) -> list[tuple[int, int]]:
    """(out, in) of each nn.Linear of a dense-connect BasicMLP (dynamics.py:412-420)."""
    sizes = [S + A] + list(hidden) + [S]
    return [(sizes[i + 1], sizes[i] + sum(sizes[:i])) for i in range(len(sizes) - 1)]


def init_model_weights(S: int, A: int, hidden, seed: int):
    """DynamicsModel.__init__ RNG order: manual_seed(seed), np.random.seed(seed), then the
    BasicMLP layers constructed in order (dynamics.py:185-196, 419)."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    out = []
    for (o, i) in basic_mlp_layer_shapes(S, A, hidden):
        lin = nn.Linear(i, o)
        out.append((lin.weight.data.clone(), lin.bias.data.clone()))
    return out


def init_ensemble_weights(S: int, A: int, hidden, num_models: int = 4, base_seed: int = 100):
    """Member k seeded base_seed + k (dynamics.py:70-79)."""
    return [init_model_weights(S, A, hidden, base_seed + k) for k in range(num_models)]


def weights_from_state_dict(sd) -> list:
    """BasicMLP state_dict ('fc_layers.{i}.weight/bias') -> [(W, b), ...]."""
    n = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("fc_layers."))
    return [(sd[f"fc_layers.{i}.weight"], sd[f"fc_layers.{i}.bias"]) for i in range(n)]


class _Member:
    """models[k]: DynamicsModel.forward(state, action, unnormalize_out=True) (dynamics.py:216-233)."""

    def __init__(self, ens: "DynamicsEnsemble", k: int):
        self._ens, self.k = ens, k

    def forward(self, state, action, unnormalize_out=True):
        if not unnormalize_out:
            raise NotImplementedError("the device path returns un-normalised deltas (the rollout's use)")
        if isinstance(state, np.ndarray):
            state = torch.from_numpy(state).float()
        if isinstance(action, np.ndarray):
            action = torch.from_numpy(action).float()
        return self._ens.device.model_forward(self.k, state, action)


class DynamicsEnsemble:
    """Reference-compatible ensemble object backed by `DeviceEnsemble`."""

    def __init__(self, state_dim: int, action_dim: int, weights, transformations, hidden_sizes=(512, 512, 512, 512),
                 device="cuda", ctx: AmxContext | None = None, feat_dim: int = 512):
        self.state_dim, self.action_dim = state_dim, action_dim
        self.num_models = len(weights)
        self.transformations = transformations
        if ctx is None:
            ctx = AmxContext(state_dim, action_dim, n_models=self.num_models, hidden=hidden_sizes[0],
                             n_hidden=len(hidden_sizes), feat_dim=feat_dim, device=device)
        self.ctx = ctx
        self.device = DeviceEnsemble(ctx, weights, transformations)
        self.models = [_Member(self, k) for k in range(self.num_models)]

    @classmethod
    def random_init(cls, state_dim, action_dim, transformations, hidden_sizes=(512, 512, 512, 512), num_models=4,
                    base_seed=100, **kw):
        w = init_ensemble_weights(state_dim, action_dim, hidden_sizes, num_models, base_seed)
        return cls(state_dim, action_dim, w, transformations, hidden_sizes, **kw)

    @classmethod
    def load_ensemble(cls, path, state_dim, action_dim, transformations, hidden_sizes=(512, 512, 512, 512), **kw):
        """dynamics.py:118-131: the saved list of {'model', 'optim'} dicts; normalizers are not
        saved by the reference and must be recomputed from the offline set."""
        sds = torch.load(path, map_location="cpu", weights_only=True)
        w = [weights_from_state_dict(d["model"]) for d in sds]
        return cls(state_dim, action_dim, w, transformations, hidden_sizes, **kw)

    @property
    def threshold(self) -> float:
        return self.device.threshold

    @threshold.setter
    def threshold(self, v: float) -> None:
        self.device.threshold = float(v)

    def compute_discrepancy(self, state, action):
        return self.device.get_action_discrepancy(state, action)

    def get_action_discrepancy(self, state, action):
        return self.device.get_action_discrepancy(state, action)

    def compute_threshold(self, states=None, actions=None):
        """dynamics.py:145-152 over the offline (s, a) rows."""
        return self.device.compute_threshold(states.to(self.ctx.device).float(), actions.to(self.ctx.device).float())
