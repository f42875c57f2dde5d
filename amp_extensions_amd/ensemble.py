"""Drop-in `DynamicsEnsemble` (milo/milo/dynamics.py:19-165) over the device ensemble.

The constructor, `load_ensemble(path)`, `save_ensemble(path)`, `compute_threshold()`,
`threshold`, `get_action_discrepancy`, `compute_discrepancy` and `models[k].forward` take the
reference's arguments and keep its semantics, so run.py's own call sequence runs unchanged
(run.py:72-78, 105, 108):

    dynamic_ensemble = DynamicsEnsemble(state_size, action_size, offline_dataset, validate_dataset,
                                        num_models=..., batch_size=..., hidden_sizes=..., transform=...,
                                        dense_connect=..., optim_args=optim_args, base_seed=args.seed,
                                        device=torch.device('cpu'))
    dynamic_ensemble.load_ensemble(ensemble_path)
    dynamic_ensemble.compute_threshold()

`device` keeps the reference's meaning (where the caller's tensors live; run.py forces the CPU,
run.py:69): results come back there.  The arithmetic always runs on the GPU (`gpu=`, default
the current HIP device) through `DeviceEnsemble` -- there is no CPU path.  The members'
parameters and optimizers are also held on the host as plain nn.Linear containers with the
reference's state-dict keys (`fc_layers.{i}.weight/bias`), so the checkpoint format written by
the reference's `save_ensemble` (a list of {'model', 'optim'}, dynamics.py:110-116) loads and
saves unchanged (torch.load with weights_only=True: tensors and plain containers only).

Inference only: ensemble training (DynamicsModel.train*, dynamics.py:236-378) is out of scope
 and `train()` raises.  The device path implements the dense-connect ReLU BasicMLP
(dynamics.py:394-433, the README command's `--dynamic_dense_connect`); other model options
raise NotImplementedError.

`as_device_ensemble(obj)` also accepts the reference's own DynamicsEnsemble object (anything
with `models[k].model.state_dict()`, `transformations` and `threshold`), so SimEnv /
BatchedSimEnv / the costs take either.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .engine import AmxContext, DeviceEnsemble

# DynamicsEnsemble's default optimizer arguments (dynamics.py:32)
DEFAULT_OPTIM_ARGS = {'optim': 'sgd', 'lr': 1e-4, 'momentum': 0.9}


def basic_mlp_layer_shapes(S: int, A: int, hidden) -> list[tuple[int, int]]:
    """(out, in) of each nn.Linear of a dense-connect BasicMLP (dynamics.py:412-420)."""
    sizes = [S + A] + list(hidden) + [S]
    return [(sizes[i + 1], sizes[i] + sum(sizes[:i])) for i in range(len(sizes) - 1)]


class BasicMLPWeights(nn.Module):
    """Host parameter container of one dense-connect BasicMLP (dynamics.py:394-420): the
    nn.Linear layers in the reference's construction order and state-dict keys.  It has no
    forward: the member's arithmetic runs on the GPU (DeviceEnsemble)."""

    def __init__(self, input_dim: int, output_dim: int, hidden_sizes):
        super().__init__()
        sizes = [input_dim] + list(hidden_sizes) + [output_dim]
        self.fc_layers = nn.ModuleList(
            nn.Linear(sizes[i] + sum(sizes[:i]), sizes[i + 1]) for i in range(len(sizes) - 1))

    def layers(self):
        return [(l.weight.data, l.bias.data) for l in self.fc_layers]

    def forward(self, x):  # pragma: no cover - guard
        raise RuntimeError("BasicMLPWeights holds parameters only; forward runs on the GPU (DynamicsEnsemble)")


def _make_optimizer(params, optim_args):
    """DynamicsModel.__init__'s optimizer (dynamics.py:199-204)."""
    if optim_args['optim'] == 'sgd':
        return torch.optim.SGD(params, lr=optim_args['lr'], momentum=optim_args['momentum'], nesterov=True)
    if optim_args['optim'] == 'adam':
        return torch.optim.Adam(params, lr=optim_args['lr'], eps=optim_args['eps'])
    raise AssertionError('Use valid optimizer')


def init_model_weights(S: int, A: int, hidden, seed: int):
    """DynamicsModel.__init__ RNG order: manual_seed(seed), np.random.seed(seed), then the
    BasicMLP layers constructed in order (dynamics.py:185-196, 419)."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    return [(w.clone(), b.clone()) for (w, b) in BasicMLPWeights(S + A, S, hidden).layers()]


def init_ensemble_weights(S: int, A: int, hidden, num_models: int = 4, base_seed: int = 100):
    """Member k seeded base_seed + k (dynamics.py:70-79)."""
    return [init_model_weights(S, A, hidden, base_seed + k) for k in range(num_models)]


def weights_from_state_dict(sd) -> list:
    """BasicMLP state_dict ('fc_layers.{i}.weight/bias') -> [(W, b), ...]."""
    n = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("fc_layers."))
    return [(sd[f"fc_layers.{i}.weight"], sd[f"fc_layers.{i}.bias"]) for i in range(n)]


class DynamicsModel:
    """models[k] of the ensemble (dynamics.py:167-392): `model` (host parameters, state-dict
    compatible), `optimizer`, `forward`, `load`, `get_state_dicts`."""

    def __init__(self, ens: "DynamicsEnsemble", k: int, state_dim: int, action_dim: int, hidden_sizes,
                 optim_args, seed: int):
        self._ens, self.k = ens, k
        self.state_dim, self.action_dim = state_dim, action_dim
        self.transform = ens.transform
        # dynamics.py:185-196: the seed, then the layers in construction order
        torch.manual_seed(seed)
        np.random.seed(seed)
        self.model = BasicMLPWeights(state_dim + action_dim, state_dim, hidden_sizes)
        self.optimizer = _make_optimizer(self.model.parameters(), optim_args)

    def forward(self, state, action, unnormalize_out=True):
        """dynamics.py:216-233: the member's Δ (un-normalised unless unnormalize_out=False),
        returned on the ensemble's `device`.  The normalised output is recovered from the
        device's un-normalised Δ as (Δ − μ_Δ)/σ_Δ (fp32, within rounding of the reference's
        raw network output)."""
        if isinstance(state, np.ndarray):
            state = torch.from_numpy(state).float()
        if isinstance(action, np.ndarray):
            action = torch.from_numpy(action).float()
        out = self._ens.engine.model_forward(self.k, state, action)
        if not unnormalize_out and self.transform:
            mu_d, sd_d = self._ens.engine.norms[4], self._ens.engine.norms[5]
            out = (out - mu_d) / sd_d
        return out.to(self._ens.device)

    def load(self, model_state_dict, optimizer_state_dict=None):
        """dynamics.py:380-386 (the device copy is refreshed by the ensemble)."""
        self.model.load_state_dict(model_state_dict)
        if optimizer_state_dict:
            self.optimizer.load_state_dict(optimizer_state_dict)

    def get_state_dicts(self):
        """dynamics.py:388-392."""
        return {'model': self.model.state_dict(), 'optim': self.optimizer.state_dict()}

    def train(self, *a, **k):
        raise NotImplementedError("dynamics-model training is out of scope (SURVEY §2); train with the reference "
                                  "and load its ensemble.pt")


def _identity_transformations(S: int, A: int):
    z_s, o_s = torch.zeros(S), torch.ones(S)
    return z_s, o_s, torch.zeros(A), torch.ones(A), z_s.clone(), o_s.clone()


def _gpu_device(gpu) -> torch.device:
    if gpu is None:
        return torch.device("cuda", torch.cuda.current_device())
    if isinstance(gpu, int):
        return torch.device("cuda", gpu)
    return torch.device(gpu)


class DynamicsEnsemble:
    """Reference-compatible DynamicsEnsemble (dynamics.py:19-165) backed by `DeviceEnsemble`."""

    def __init__(self, state_dim, action_dim, train_dataset, validate_dataset=None, num_models=4, batch_size=256,
                 hidden_sizes=[512, 512], use_resnet=False, dense_connect=True, activation='relu', transform=True,
                 optim_args=DEFAULT_OPTIM_ARGS, device=torch.device('cpu'), base_seed=100, num_workers=1, *,
                 gpu=None, ctx: AmxContext | None = None, feat_dim: int = 512, gemm: str = "f16x3"):
        """The reference's arguments (dynamics.py:20-35).  `train_dataset` supplies the
        normalizers (`get_transformations`, datasets.py:23-43) and the rows compute_threshold
        scans; `validate_dataset`, `batch_size` and `num_workers` only configure training in the
        reference and are kept for the call's shape.  Extensions (keyword-only): `gpu` (the HIP
        device the arithmetic runs on), `ctx` (share an AmxContext), `feat_dim` (the context's
        RFF width), `gemm` (DeviceEnsemble's GEMM path)."""
        if use_resnet or not dense_connect or activation != 'relu':
            raise NotImplementedError("the device ensemble implements the dense-connect ReLU BasicMLP "
                                      "(dynamics.py:394-433; run.py's --dynamic_dense_connect): got "
                                      f"use_resnet={use_resnet}, dense_connect={dense_connect}, activation={activation!r}")
        hidden_sizes = list(hidden_sizes)
        if len(set(hidden_sizes)) != 1:
            raise NotImplementedError(f"the device ensemble needs equal hidden widths, got {hidden_sizes}")
        self.state_dim, self.action_dim = state_dim, action_dim
        self.train_dataset, self.validate_dataset = train_dataset, validate_dataset
        self.batch_size = batch_size
        self.transformations = train_dataset.get_transformations(device) if transform else None
        self.num_models = num_models
        self.transform = transform
        self.device = device if isinstance(device, torch.device) else torch.device(device)
        self.base_seed = base_seed
        self.hidden_sizes = hidden_sizes
        self.models = [DynamicsModel(self, k, state_dim, action_dim, hidden_sizes, optim_args, base_seed + k)
                       for k in range(num_models)]
        if ctx is None:
            ctx = AmxContext(state_dim, action_dim, n_models=num_models, hidden=hidden_sizes[0],
                             n_hidden=len(hidden_sizes), feat_dim=feat_dim, device=_gpu_device(gpu))
        self.ctx = ctx
        self.engine = DeviceEnsemble(ctx, [m.model.layers() for m in self.models], self._norms(), gemm=gemm)
        self._set_member_transformations()
        self.threshold = 0.0

    # ---- construction helpers (extensions) --------------------------------------------------
    @classmethod
    def from_weights(cls, state_dim, action_dim, weights, transformations, hidden_sizes=(512, 512, 512, 512),
                     threshold: float = 0.0, **kw):
        """An ensemble over given per-member [(W, b), ...] weights (nn.Linear layout) and the
        six normalizer vectors (datasets.py:23-43), without an offline dataset."""
        ds = _Transformations(transformations)
        ens = cls(state_dim, action_dim, ds, None, num_models=len(weights), hidden_sizes=list(hidden_sizes), **kw)
        for m, w in zip(ens.models, weights):
            with torch.no_grad():
                for lin, (W, b) in zip(m.model.fc_layers, w):
                    lin.weight.copy_(torch.as_tensor(W)), lin.bias.copy_(torch.as_tensor(b))
        ens._upload()
        ens.threshold = threshold
        return ens

    @classmethod
    def random_init(cls, state_dim, action_dim, transformations, hidden_sizes=(512, 512, 512, 512), num_models=4,
                    base_seed=100, **kw):
        """The reference's seeded init (member k: base_seed + k) with given normalizers."""
        return cls(state_dim, action_dim, _Transformations(transformations), None, num_models=num_models,
                   hidden_sizes=list(hidden_sizes), base_seed=base_seed, **kw)

    @classmethod
    def from_reference(cls, ref, **kw):
        """Convert the reference's DynamicsEnsemble object (its members' BasicMLP state dicts,
        transformations and threshold)."""
        sds = [m.model.state_dict() for m in ref.models]
        w = [weights_from_state_dict(sd) for sd in sds]
        S, A = ref.state_dim, ref.action_dim
        hidden = [W.shape[0] for (W, _) in w[0][:-1]]
        tr = ref.transformations if getattr(ref, "transform", True) and ref.transformations is not None \
            else _identity_transformations(S, A)
        return cls.from_weights(S, A, w, tr, hidden_sizes=hidden, threshold=float(ref.threshold), **kw)

    # ---- the reference surface -------------------------------------------------------------
    def _norms(self):
        if self.transformations is None:
            return _identity_transformations(self.state_dim, self.action_dim)
        return tuple(torch.as_tensor(x).detach().float().cpu() for x in self.transformations)

    def _set_member_transformations(self):
        if self.transform:  # dynamics.py:128-131
            for m in self.models:
                (m.state_mean, m.state_scale, m.action_mean, m.action_scale, m.diff_mean,
                 m.diff_scale) = self.transformations

    def _upload(self):
        self.engine.set_weights([m.model.layers() for m in self.models])

    @property
    def threshold(self) -> float:
        return self.engine.threshold

    @threshold.setter
    def threshold(self, v) -> None:
        self.engine.threshold = float(v)

    def train(self, *a, **k):
        raise NotImplementedError("ensemble training is out of scope (SURVEY §2); train with the reference and "
                                  "load its ensemble.pt with load_ensemble")

    def save_ensemble(self, save_path):
        """dynamics.py:110-116: a list of {'model', 'optim'} state dicts."""
        torch.save([m.get_state_dicts() for m in self.models], save_path)

    def load_ensemble(self, state_dict_path):
        """dynamics.py:118-131: the members' model (and optimizer) state dicts from the list
        save_ensemble wrote, then the dataset's transformations; the device weights are
        refreshed in place.  Loaded with the weights-only unpickler (tensors and plain
        containers; anything else in the file is refused)."""
        state_dicts = torch.load(state_dict_path, map_location="cpu", weights_only=True)
        assert len(state_dicts) == len(self.models)
        print("loading ensemble")
        for model, state_dict in zip(self.models, state_dicts):
            model.load(state_dict['model'], state_dict['optim'])
        print("Done loading ensemble")
        self._set_member_transformations()
        self._upload()

    def discrepancy_device(self, state, action) -> torch.Tensor:
        """The per-row max pairwise disagreement, left on the GPU (the costs' input)."""
        return self.engine.get_action_discrepancy(torch.as_tensor(state), torch.as_tensor(action))

    def compute_discrepancy(self, state, action):
        """dynamics.py:134-143: max over member pairs of ‖pred_i − pred_j‖₂, on the CPU."""
        return self.discrepancy_device(state, action).to(torch.device('cpu'))

    def get_action_discrepancy(self, state, action):
        """dynamics.py:154-165 (float32 inputs; the result on the CPU as the reference's)."""
        return self.compute_discrepancy(state, action)

    def compute_threshold(self, states=None, actions=None):
        """dynamics.py:145-152: the max disagreement over the whole offline (train) dataset.
        (states, actions) may be given explicitly (extension; then the threshold is returned)."""
        explicit = states is not None
        if not explicit:
            ds = self.train_dataset
            if hasattr(ds, "states") and hasattr(ds, "actions"):
                states, actions = ds.states, ds.actions
            else:
                rows = [ds[i] for i in range(len(ds))]
                states = torch.stack([r[0] for r in rows])
                actions = torch.stack([r[1] for r in rows])
        dev = self.ctx.device
        self.engine.compute_threshold(torch.as_tensor(states).to(dev).float(), torch.as_tensor(actions).to(dev).float())
        return self.threshold if explicit else None


class _Transformations:
    """A stand-in train_dataset that only supplies get_transformations (from_weights / random_init)."""

    def __init__(self, tr):
        self._tr = tuple(torch.as_tensor(x).detach().float().cpu() for x in tr)

    def get_transformations(self, device=None):
        return tuple(x.to(device) if device is not None else x for x in self._tr)

    def __len__(self):
        return 0


def as_device_ensemble(ens) -> DeviceEnsemble:
    """The DeviceEnsemble behind `ens`: this package's DynamicsEnsemble, a DeviceEnsemble, or
    the reference's DynamicsEnsemble object (converted once and cached on it; run.py loads the
    weights before it builds the env, run.py:78-120)."""
    if isinstance(ens, DeviceEnsemble):
        return ens
    if isinstance(ens, DynamicsEnsemble):
        return ens.engine
    conv = getattr(ens, "_amx_ensemble", None)
    if conv is None:
        if not (hasattr(ens, "models") and hasattr(ens, "threshold")):
            raise TypeError(f"expected a DynamicsEnsemble, got {type(ens).__name__}")
        conv = DynamicsEnsemble.from_reference(ens)
        try:
            ens._amx_ensemble = conv
        except AttributeError:
            pass
    return conv.engine
