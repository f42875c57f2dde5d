"""CPU-only checks: the C-ABI library builds/loads and exports every declared symbol, the
host-side layout/packing logic, and the ABI's argument validation (no kernel launches)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from amp_extensions_amd import _build, _native
from amp_extensions_amd import synthetic as syn
from amp_extensions_amd.ensemble import basic_mlp_layer_shapes, init_ensemble_weights, weights_from_state_dict
from amp_extensions_amd.humanoid import TerminationConfig, FALL_BODIES


@pytest.fixture(scope="module")
def lib():
    path = _build.build(verbose=False)
    return _native.load(path)


def test_library_exports_every_header_symbol(lib):
    syms = _native.header_symbols()
    assert len(syms) >= 20
    raw = ctypes.CDLL(_build.LIB_PATH)
    for s in syms:
        assert hasattr(raw, s), s
    # the Python binding declares exactly the header's functions
    assert sorted(_native.SIGNATURES) == sorted(syms)


def test_library_is_gfx950_code_object():
    data = open(_build.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_abi_version_and_errors(lib):
    assert lib.amx_abi_version() == _native.ABI_VERSION == 2
    # bad dims are refused without touching the GPU
    assert not lib.amx_create(0, 226, 28, 9, 512, 4, 512)   # > AMX_MAX_MODELS
    assert b"bad dims" in lib.amx_last_error()
    assert not lib.amx_create(0, 226, 28, 4, 500, 4, 512)   # hidden not a multiple of 128
    # null-context calls fail with AMX_E_INVAL and a message
    rc = lib.amx_gemm_bias_act(None, 1, 128, 128, 32, None, 32, 0, None, 32, 0, None, 0, None, 128, 0, 0, 1, None)
    assert rc == -1
    rc = lib.amx_step(None, None, 226, 0, None, None, None, None, None, None, None, 0, None, 1, None)
    assert rc == -1 and b"amx_step" in lib.amx_last_error()


def test_round4_entry_points_validate_without_gpu(lib):
    """The round-4/5 NPG / noise entry points refuse bad arguments before any launch, and the CG
    tail's workspace size is pure host arithmetic (P + ceil(P / 64) doubles)."""
    assert lib.amx_npg_cg_tail_work(8616) == 8616 + 135
    assert lib.amx_npg_cg_tail_work(64) == 64 + 1
    assert lib.amx_npg_curvature(None, None, 10, 4, None, None) == -1
    assert lib.amx_npg_apply_step(None, 10, 4, None, None, None, 0, 0.0, 0.1, -2.0, None, None, None) == -1
    assert b"amx_npg_apply_step" in lib.amx_last_error()
    assert lib.amx_npg_cg_tail(None, None, 1, 10, 4, None, 0.0, 0.0, None, None, None, None, None, None, None,
                               None, None) == -1
    assert lib.amx_npg_pass_ex(None, 1, 64, None, 1, 197, None, 1, 36, None, None, None, 32, None, None, None,
                               None) == -1
    # round 6: the CG tail's two launches separately, and the Fisher-vector pass with the step folded in
    assert lib.amx_npg_cg_reduce(None, None, 1, 10, 4, None, 0.0, None, None, None, None, None) == -1
    assert b"amx_npg_cg_reduce" in lib.amx_last_error()
    assert lib.amx_npg_cg_xrp(None, 10, 0.0, None, None, None, None, None, None, None, None, None) == -1
    assert b"amx_npg_cg_xrp" in lib.amx_last_error()
    assert lib.amx_npg_pass_cg(None, 64, None, 1, 197, None, 32, None, None, 0.0, None, None, None, None, None, None,
                               None, None, None, None) == -1
    assert b"amx_npg_pass_cg" in lib.amx_last_error()


def test_dense_layer_shapes_match_basicmlp():
    # dynamics.py:412-420: input of layer i = concat of all previous widths
    assert basic_mlp_layer_shapes(226, 28, [512] * 4) == [(512, 254), (512, 766), (512, 1278), (512, 1790),
                                                          (226, 2302)]
    macs = sum(o * i for o, i in basic_mlp_layer_shapes(226, 28, [512] * 4))
    assert macs == 2613308
    assert sum(o * i for o, i in basic_mlp_layer_shapes(197, 36, [512] * 4)) == 2499405


def test_init_matches_oracle_rng_order():
    from oracle import milo_ref as R
    a = init_ensemble_weights(226, 28, [64] * 4, 2, 100)
    b = R.init_ensemble_weights(226, 28, [64] * 4, 2, 100)
    for ma, mb in zip(a, b):
        for (wa, ba), (wb, bb) in zip(ma, mb):
            assert torch.equal(wa, wb) and torch.equal(ba, bb)


def test_state_dict_roundtrip():
    w = init_ensemble_weights(20, 4, [16, 16], 1, 5)[0]
    sd = {f"fc_layers.{i}.weight": W for i, (W, _) in enumerate(w)}
    sd.update({f"fc_layers.{i}.bias": b for i, (_, b) in enumerate(w)})
    back = weights_from_state_dict(sd)
    assert all(torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]) for x, y in zip(back, w))


def test_termination_tables():
    ids, shapes, p0, p1 = TerminationConfig().tables()
    assert tuple(ids) == FALL_BODIES and len(ids) == 13
    assert shapes.count(0) == 5 and shapes.count(1) == 8  # 5 spheres, 8 capsules (humanoid3d.txt)
    assert max(9 * b + 5 for b in ids) < 197  # every index valid in both layouts


def test_synthetic_reset_table_starts_standing():
    t = syn.reset_table(512, 226, 1)
    for b in FALL_BODIES:
        assert (t[:, 9 * b + 2] >= 0.2).all()
    s, a, s2 = syn.offline(64, 197, 36, 0)
    assert s.shape == (64, 197) and a.shape == (64, 36)
    assert syn.expert(32, 197).shape == (32, 394)


def test_product_package_never_imports_oracle():
    root = os.path.dirname(_build.PKG_DIR)
    for dp, _, fs in os.walk(_build.PKG_DIR):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f
    assert os.path.isdir(os.path.join(root, "oracle"))


# ---- on-disk trajectory databases (milo/milo/utils.py:222-305) vs the reference (G10) -------
def _g10_dbs():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "make_golden", os.path.join(os.path.dirname(__file__), "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg.g10_dbs()


def test_db_loaders_match_reference(golden, tmp_path):
    import numpy as np
    import torch
    from amp_extensions_amd import datasets as D
    g = golden("g10_db.npz")
    offline, expert = _g10_dbs()
    fo, fe = str(tmp_path / "offline.pt"), str(tmp_path / "expert.pt")
    torch.save(offline, fo)
    torch.save(expert, fe)
    for tag, kw in (("amp", dict(imitate_amp=True)), ("rew", dict(imitate_amp=False)), ("n2", dict(num_trajs=2))):
        s, a, s2 = D.get_db_mjrl(fo, verbose=False, **kw)
        for x, k in ((s, "s"), (a, "a"), (s2, "s2")):
            assert x.dtype == torch.float32
            np.testing.assert_array_equal(x.numpy(), g[f"db_{tag}_{k}"])
    es, es2 = D.get_db_mjrl(fe, expert=True)
    np.testing.assert_array_equal(es.numpy(), g["ex_s"])
    np.testing.assert_array_equal(es2.numpy(), g["ex_s2"])
    p = D.get_paths_mjrl(fo, idx=1)
    assert len(p) == 1
    np.testing.assert_array_equal(p[0]["observations"], g["paths_idx1_obs"])
    np.testing.assert_array_equal(p[0]["actions"], g["paths_idx1_act"])
    p = D.get_paths_mjrl(fe, expert=True)
    np.testing.assert_array_equal(np.concatenate([q["next_observation"] for q in p]), g["paths_ex_nobs"])
    x = D.convert_to_veltopos(fo, vel_offset=136, dt=1 / 30)
    np.testing.assert_array_equal(np.concatenate([t["episode"][0] for t in x]), g["v2p_offline"])
    x = D.convert_to_veltopos(fe, is_expert=True, vel_offset=136, dt=1 / 30)
    np.testing.assert_array_equal(np.concatenate([t["episode"] for t in x]), g["v2p_expert"])
    # idx on get_db_mjrl selects one trajectory (the reference iterates that dict's keys)
    s, a, s2 = D.get_db_mjrl(fo, idx=2, verbose=False)
    T = offline[2]["episode"][1].shape[0]
    assert s.shape == (T, offline[2]["episode"][0].shape[1]) and a.shape[0] == T


def test_db_loader_refuses_arbitrary_callables(tmp_path):
    import pickle

    import pytest
    import torch
    from amp_extensions_amd import datasets as D

    class Evil:
        def __reduce__(self):
            return (print, ("should not run",))

    f = tmp_path / "evil.pt"
    torch.save([{"episode": Evil()}], str(f), pickle_module=pickle)
    with pytest.raises(Exception):
        D.load_db(str(f))


def test_npg_pack_unpack_roundtrip():
    """DeviceNPG's flat parameter order is the reference's (MLP.trainable_params)."""
    from amp_extensions_amd.npg import pack_policy, unpack_policy
    from amp_extensions_amd.policy import init_mlp_policy_params
    from oracle import milo_ref as R
    layers, ls = init_mlp_policy_params(226, 28, (32, 32), seed=100, init_log_std=-0.25)
    flat = pack_policy(layers, ls)
    shapes = R.policy_param_shapes(226, 28, (32, 32))
    assert flat.size == sum(int(np.prod(s)) for s in shapes)
    l2, ls2 = unpack_policy(flat, 226, 28)
    for (W, b), (W2, b2) in zip(layers, l2):
        assert torch.equal(W, W2) and torch.equal(b, b2)
    assert torch.equal(ls, ls2)


# ---- a1: the product's normalizers (amp_extensions_amd.datasets) vs the reference (G7) -----
def test_product_transformations_match_reference(golden):
    """AmpDataset.get_transformations (milo/milo/datasets.py:23-43) as the product computes it
    (the normalizers DeviceEnsemble uploads) equals the reference's own output bit for bit."""
    from amp_extensions_amd.datasets import AmpDataset, get_transformations
    g = golden("g7_transformations.npz")
    torch.set_num_threads(1)  # the fixture was generated single-threaded
    rs = np.random.RandomState(int(g["seed"]))
    n = int(g["n"])
    s = 0.5 * rs.randn(n, 226)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, 28)
    s2 = s + 0.01 * rs.randn(n, 226)
    st, at, s2t = (torch.from_numpy(x).float() for x in (s, a, s2))
    keys = ["mu_s", "sd_s", "mu_a", "sd_a", "mu_d", "sd_d"]
    for out in (get_transformations(st, at, s2t), AmpDataset(st, at, s2t).get_transformations()):
        for k, v in zip(keys, out):
            assert v.dtype == torch.float32
            np.testing.assert_array_equal(v.numpy(), g[k], err_msg=k)


def test_motion_bundle_matches_reference_data(golden):
    """The packaged character + spinkick clip (amp_extensions_amd/data, tools/pack_motion.py)
    holds the reference's data files (the G12 fixture was read from them)."""
    import json
    from amp_extensions_amd.motion import ReferenceMotion
    g = golden("g12_motion.npz")
    with np.load(ReferenceMotion.DEFAULT_BUNDLE, allow_pickle=False) as z:
        assert json.loads(str(z["character_json"])) == json.loads(str(g["character_json"]))
        np.testing.assert_array_equal(z["frames"], g["frames"])
        assert str(z["loop"]) == str(g["loop"])


def test_deepmimic_arg_file_parsing_and_reset_args(tmp_path):
    """SimEnv's host side of the run.py construction (sim_env.py:76-99): DeepMimic's ArgParser
    rules (comment lines and tokens skipped, the first occurrence of a key wins, data paths
    resolved from the package root), the ctrl flags and BodyDefs read into the termination
    config, and reset_args: defaults filled in, the AddNoise options accepted (applied on the
    device, tests/test_gpu_motion.py), NaN amounts refused."""
    from amp_extensions_amd import sim_env as SE
    from test_gpu_simenv_dropin import RUN_PY_RESET_ARGS, write_deepmimic_tree
    args = write_deepmimic_tree(str(tmp_path))
    table = SE.parse_deepmimic_args(args)
    assert table["motion_file"] == ["data/motions/humanoid3d_spinkick.txt"]  # first occurrence wins
    assert "model_files" not in table and table["time_lim_min"] == ["0.5"]
    assert table["fall_contact_bodies"] == [str(i) for i in FALL_BODIES]
    assert SE._arg_file(table, "motion_file", args) == os.path.join(str(tmp_path), "data/motions/humanoid3d_spinkick.txt")
    cfg = SE.termination_from_args(args, 300, False)
    assert cfg.record_world_root_pos is False and cfg.record_all_world is False
    assert abs(cfg.sampling_rate - 1.0 / 30) < 1e-15 and len(cfg.body_defs) == 15
    ra = SE.check_reset_args({"custom_time": True, "time_max": 0.5})
    assert ra["resolve"] is True and ra["time_max"] == 0.5 and ra["radian"] == 0
    assert SE.check_reset_args(RUN_PY_RESET_ARGS)["interp"] == 1.0
    assert SE.check_reset_args(dict(RUN_PY_RESET_ARGS, vel_noise=True, knee_rot=True, interp=0.3))
    ra = SE.check_reset_args(dict(RUN_PY_RESET_ARGS, noise_max=0.1, radian=0.2))  # AddNoise (device)
    assert ra["noise_max"] == 0.1 and ra["radian"] == 0.2
    with pytest.raises(ValueError):
        SE.check_reset_args(dict(RUN_PY_RESET_ARGS, radian=float("nan")))
    with pytest.raises(FileNotFoundError):
        SE.motion_from_args(None, str(tmp_path / "missing_args.txt"))


def test_host_policy_noise_matches_numpy_legacy_stream(lib):
    """amx_mt_seed / amx_mt_policy_noise (the sampler's per-lane policy noise) reproduce numpy's
    legacy RandomState bit for bit as mjrl MLP.get_action draws it after np.random.seed(s)
    (gaussian_mlp.py:99-102: np.random.uniform(), then np.random.randn(A), per step), carried
    across calls (the polar method's cached normal included: odd A), for the full seed range."""
    for A in (36, 7):
        L, K = 6, 5
        st = np.zeros((L, _native.AMX_MT_STATE_BYTES), np.uint8)
        slots = np.array([0, 2, 5, 3], np.int32)
        seeds = np.array([12345, 12345 + 100 * 3 + 7, 0, 2 ** 32 - 1], np.uint32)
        assert lib.amx_mt_seed(st.ctypes.data, L, slots.ctypes.data, seeds.ctypes.data, 4) == 0
        rss = [np.random.RandomState(int(x)) for x in seeds]
        out = np.full((K, L, A), np.nan)
        for rep in range(3):
            sub = slots[rep % 2:]  # not every lane advances in every chunk
            assert lib.amx_mt_policy_noise(st.ctypes.data, L, sub.ctypes.data, sub.size, K, A, out.ctypes.data,
                                           L * A, A) == 0
            for lane in sub:
                i = list(slots).index(lane)
                want = np.empty((K, A))
                for k in range(K):
                    rss[i].uniform()
                    want[k] = rss[i].randn(A)
                np.testing.assert_array_equal(out[:, lane], want)
    bad = np.array([L], np.int32)
    assert lib.amx_mt_seed(st.ctypes.data, L, bad.ctypes.data, seeds.ctypes.data, 1) != 0


def test_host_policy_noise_many_lanes(lib):
    """Chunks of >= 32 lanes are split over host threads: every lane's stream stays
    bit-identical to numpy's legacy RandomState over repeated calls, independent of how the lanes
    were dealt to the threads."""
    L, K, A = 300, 4, 36
    st = np.zeros((L, _native.AMX_MT_STATE_BYTES), np.uint8)
    slots = np.arange(L, dtype=np.int32)
    seeds = (12345 + 7 * np.arange(L)).astype(np.uint32)
    assert lib.amx_mt_seed(st.ctypes.data, L, slots.ctypes.data, seeds.ctypes.data, L) == 0
    rss = [np.random.RandomState(int(x)) for x in seeds]
    out = np.full((K, L, A), np.nan)
    for rep in range(4):
        assert lib.amx_mt_policy_noise(st.ctypes.data, L, slots.ctypes.data, L, K, A, out.ctypes.data, L * A, A) == 0
        for lane in (0, 1, 31, 32, 150, 299):
            want = np.empty((K, A))
            for k in range(K):
                rss[lane].uniform()
                want[k] = rss[lane].randn(A)
            np.testing.assert_array_equal(out[:, lane], want)
        for lane in set(range(L)) - {0, 1, 31, 32, 150, 299}:  # keep the reference streams in step
            for k in range(K):
                rss[lane].uniform()
                rss[lane].randn(A)


def test_reference_checkpoint_loads_into_host_members(golden, golden_path):
    """G13's ensemble.pt (written by the reference's save_ensemble, dynamics.py:110-116) loads
    with the weights-only unpickler into the drop-in members' host containers (the reference's
    state-dict keys) and into run.py's default optimizer (Adam) with its state; the seeded init
    of the containers draws what DynamicsModel.__init__ draws (oracle restatement)."""
    from oracle import milo_ref as R
    from amp_extensions_amd.ensemble import BasicMLPWeights, _make_optimizer, init_model_weights
    g = golden("g13_ensemble_ckpt.npz")
    hidden = [int(x) for x in g["hidden"]]
    S, A = 226, 28
    sds = torch.load(golden_path("g13_ensemble.pt"), map_location="cpu", weights_only=True)
    assert isinstance(sds, list) and len(sds) == 4 and all(set(d) == {"model", "optim"} for d in sds)
    for k, d in enumerate(sds):
        m = BasicMLPWeights(S + A, S, hidden)
        m.load_state_dict(d["model"])
        opt = _make_optimizer(m.parameters(), {"optim": str(g["optim"]), "lr": float(g["lr"]), "eps": float(g["eps"])})
        opt.load_state_dict(d["optim"])
        st = opt.state_dict()["state"]
        assert len(st) == 2 * (len(hidden) + 1) and all("exp_avg" in v for v in st.values())
        for (W, b), (W2, b2) in zip(m.layers(), weights_from_state_dict(d["model"])):
            assert torch.equal(W, W2) and torch.equal(b, b2)
        for (W, b), (Wr, br) in zip(init_model_weights(S, A, hidden, 100 + k), R.init_model_weights(S, A, hidden, 100 + k)):
            assert torch.equal(W, Wr) and torch.equal(b, br)


def test_sampler_free_lanes_member_blocks():
    """The sampler's idle-lane pool: one list without member blocks; with blocks of Bq lanes
    trajectory j takes a lane of block j mod M (the member its reset selects), -1 when that
    block is full, and a freed lane returns to its own block."""
    from amp_extensions_amd.sampler import _FreeLanes
    f = _FreeLanes(5, 4, 0)
    assert [f.take(j) for j in range(1, 6)] == [0, 1, 2, 3, 4] and not f and f.take(1) == -1
    f.put(3)
    assert f and f.take(7) == 3
    g = _FreeLanes(8, 4, 2)
    got = [g.take(j) for j in (1, 2, 3, 4, 5, 9)]
    assert got == [2, 4, 6, 0, 3, -1]
    assert g.take(8) == 1 and g.take(4) == -1
    g.put(3)
    assert g.take(13) == 3
