"""run.py's dynamics-ensemble call sequence, as written, on the reference's own checkpoint.

G13 (tests/golden/make_golden.py) is an `ensemble.pt` written by the reference's
`DynamicsEnsemble.save_ensemble` (milo/milo/dynamics.py:110-116: a list of {'model', 'optim'},
Adam state included) after one optimizer step per member, plus the reference's outputs after
run.py:72-78 (construct + load_ensemble) and :108 (compute_threshold()).  Here the same lines
run against the drop-in `amp_extensions_amd.ensemble.DynamicsEnsemble` with the GPU doing the
arithmetic, then run.py:120 builds the env from it.  Tolerances: member forwards 2e-5 of
max(1, |ref|) (fp32 GEMM order), disagreement / threshold rel 1e-4."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R
from test_gpu_simenv_dropin import RUN_PY_RESET_ARGS, write_deepmimic_tree

pytestmark = pytest.mark.gpu
S, A = 226, 28


def synthetic_offline(n, seed):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


def _rel(x, ref):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return float((np.abs(x - ref) / np.maximum(1.0, np.abs(ref))).max())


@pytest.fixture(scope="module")
def run_py(golden, golden_path):
    """run.py:42-43 (AmpDataset of the offline set), :54-57 (optim_args), :68-78, :108."""
    from amp_extensions_amd.datasets import AmpDataset
    from amp_extensions_amd.ensemble import DynamicsEnsemble
    g = golden("g13_ensemble_ckpt.npz")
    s, a, s2 = synthetic_offline(int(g["n_offline"]), int(g["offline_seed"]))
    device = torch.device("cpu")  # run.py:69 forces the CPU
    offline_dataset = AmpDataset(torch.from_numpy(s).float(), torch.from_numpy(a).float(),
                                 torch.from_numpy(s2).float(), device)
    validate_dataset = None
    optim_args = {"optim": str(g["optim"]), "lr": float(g["lr"]), "eps": float(g["eps"])}
    hidden = [int(x) for x in g["hidden"]]
    ensemble_path = golden_path("g13_ensemble.pt")

    dynamic_ensemble = DynamicsEnsemble(S, A, offline_dataset, validate_dataset,
                                        num_models=4,
                                        batch_size=256, hidden_sizes=hidden,
                                        transform=True,
                                        dense_connect=True, optim_args=optim_args,
                                        base_seed=int(g["base_seed"]), device=device)
    dynamic_ensemble.load_ensemble(ensemble_path)
    dynamic_ensemble.compute_threshold()
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    return g, dynamic_ensemble, R.load_ensemble_weights(ensemble_path), norms


def test_run_py_sequence_matches_reference(run_py):
    g, ens, _, _ = run_py
    assert abs(ens.threshold - float(g["threshold"])) <= 1e-4 * abs(float(g["threshold"]))
    qs, qa = torch.from_numpy(g["query_s"]), torch.from_numpy(g["query_a"])
    for k, m in enumerate(ens.models):
        out = m.forward(qs, qa)
        assert out.device == torch.device("cpu")  # returned where the caller's device says (run.py:69)
        assert _rel(out.numpy(), g["preds"][k]) <= 2e-5
        assert _rel(m.forward(qs, qa, unnormalize_out=False).numpy(), g["preds_norm"][k]) <= 2e-5
    d = ens.get_action_discrepancy(qs, qa)
    assert d.device == torch.device("cpu")  # dynamics.py:143
    np.testing.assert_allclose(d.numpy(), g["disc"], rtol=1e-4, atol=1e-4 * float(np.abs(g["disc"]).max()))


def test_loaded_state_is_the_files(run_py, golden_path):
    """load_ensemble took every member's model AND optimizer state from the file."""
    _, ens, _, _ = run_py
    sds = torch.load(golden_path("g13_ensemble.pt"), map_location="cpu", weights_only=True)
    for m, sd in zip(ens.models, sds):
        for k, v in sd["model"].items():
            assert torch.equal(m.model.state_dict()[k], v), k
        mine, ref = m.optimizer.state_dict(), sd["optim"]
        assert mine["param_groups"] == ref["param_groups"]
        for i, st in ref["state"].items():
            for k, v in st.items():
                assert torch.equal(torch.as_tensor(mine["state"][i][k]), torch.as_tensor(v)), (i, k)


def test_save_ensemble_round_trip(run_py, tmp_path):
    """save_ensemble writes the reference's format; loading it into a second ensemble gives
    bit-identical device results."""
    from amp_extensions_amd.ensemble import DynamicsEnsemble
    g, ens, _, _ = run_py
    p = str(tmp_path / "ensemble.pt")
    ens.save_ensemble(p)
    sds = torch.load(p, map_location="cpu", weights_only=True)
    assert len(sds) == 4 and all(set(d) == {"model", "optim"} for d in sds)
    other = DynamicsEnsemble(S, A, ens.train_dataset, None, num_models=4, hidden_sizes=[int(x) for x in g["hidden"]],
                             optim_args={"optim": "adam", "lr": 1e-3, "eps": 1e-8}, base_seed=7, ctx=ens.ctx)
    qs, qa = torch.from_numpy(g["query_s"]), torch.from_numpy(g["query_a"])
    before = other.models[0].forward(qs, qa)
    other.load_ensemble(p)
    for k in range(4):
        assert torch.equal(other.models[k].forward(qs, qa), ens.models[k].forward(qs, qa))
    assert not torch.equal(before, other.models[0].forward(qs, qa))  # the in-place refresh took


def test_run_py_env_steps_with_loaded_ensemble(run_py, tmp_path):
    """run.py:113-120: the env built from the loaded ensemble steps as the oracle SimEnv with
    the file's weights (per-step parity from the oracle's state, done flags exact)."""
    import amp_extensions_amd as amx
    g, dynamic_ensemble, ens_w, norms = run_py
    args = write_deepmimic_tree(str(tmp_path))
    mb_env = amx.SimEnv(deepmimic_args=args, dynamic_ensemble=dynamic_ensemble, reset_args=RUN_PY_RESET_ARGS)
    mb_env.seed_env(21)
    ref = R.SimEnvRef(ens_w, norms, horizon=300)
    acts = np.random.RandomState(22).randn(120, A) * np.exp(-0.25)
    o = mb_env.reset()
    ref.reset(o.copy())
    worst = 0.0
    for t in range(acts.shape[0]):
        mb_env.set_observation(ref.ob.copy())
        no, r, d, info = mb_env.step(acts[t].copy())
        rno, _, rd, _ = ref.step(acts[t].copy())
        assert r == 0 and info == {} and d == rd, t
        worst = max(worst, _rel(no, rno))
        if d:
            o = mb_env.reset()
            ref.reset(o.copy())
    assert worst <= 2e-5, worst


class _RefMember:
    def __init__(self, model):
        self.model = model


class _ReferenceLikeEnsemble:
    """The attributes of the reference's DynamicsEnsemble object that a conversion reads
    (dynamics.py:54-80): state/action dims, models[k].model (a BasicMLP), transform,
    transformations, threshold."""

    def __init__(self, S, A, models, transformations, threshold):
        self.state_dim, self.action_dim = S, A
        self.models = [_RefMember(m) for m in models]
        self.transform, self.transformations, self.threshold = True, transformations, threshold


def test_reference_ensemble_object_drops_in(run_py, tmp_path):
    """A reference DynamicsEnsemble object (as run.py would hand over after its own
    load_ensemble) is accepted by SimEnv and the costs, and computes what the drop-in does."""
    import amp_extensions_amd as amx
    from amp_extensions_amd.ensemble import BasicMLPWeights, as_device_ensemble
    g, ens, _, norms = run_py
    hidden = [int(x) for x in g["hidden"]]
    models = []
    for m in ens.models:
        b = BasicMLPWeights(S + A, S, hidden)
        b.load_state_dict(m.model.state_dict())
        models.append(b)
    ref_obj = _ReferenceLikeEnsemble(S, A, models, norms, ens.threshold)
    dev = as_device_ensemble(ref_obj)
    assert as_device_ensemble(ref_obj) is dev  # converted once
    qs = torch.from_numpy(g["query_s"]).cuda()
    qa = torch.from_numpy(g["query_a"]).cuda()
    assert torch.equal(dev.get_action_discrepancy(qs, qa), ens.engine.get_action_discrepancy(qs, qa))
    assert dev.threshold == ens.threshold
    args = write_deepmimic_tree(str(tmp_path))
    env = amx.SimEnv(deepmimic_args=args, dynamic_ensemble=ref_obj, reset_args=RUN_PY_RESET_ARGS, seed=3)
    env2 = amx.SimEnv(deepmimic_args=args, dynamic_ensemble=ens, reset_args=RUN_PY_RESET_ARGS, seed=3)
    o, o2 = env.reset(), env2.reset()
    np.testing.assert_array_equal(o, o2)
    a = np.random.RandomState(4).randn(A) * 0.5
    n1, _, d1, _ = env.step(a.copy())
    n2, _, d2, _ = env2.step(a.copy())
    np.testing.assert_array_equal(n1, n2)
    assert d1 == d2
    s, _, s2 = synthetic_offline(512, 3)
    expert = torch.cat([torch.from_numpy(s).float(), torch.from_numpy(s2).float()], 1)
    cost = amx.RBFLinearCost(expert, feature_dim=512, lambda_b=0.0025, seed=100, ctx=ens.ctx)
    ps, pa, ps2 = [torch.from_numpy(x).float() for x in synthetic_offline(96, 4)]
    cost.fit_cost(torch.cat([ps, ps2], 1))
    c1, _ = cost.get_bonus_costs(ps, pa, ref_obj, next_states=ps2)
    c2, _ = cost.get_bonus_costs(ps, pa, ens, next_states=ps2)
    assert torch.equal(c1, c2)


def test_unsupported_model_options_raise(run_py):
    from amp_extensions_amd.ensemble import DynamicsEnsemble
    _, ens, _, _ = run_py
    for kw in (dict(use_resnet=True), dict(dense_connect=False), dict(activation="tanh")):
        with pytest.raises(NotImplementedError):
            DynamicsEnsemble(S, A, ens.train_dataset, None, hidden_sizes=[32, 32], ctx=ens.ctx, **kw)
    with pytest.raises(NotImplementedError):
        ens.train(1)
