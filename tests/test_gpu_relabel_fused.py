"""The relabel tail in one launch (amx_mmd_relabel) and the feature message
(amx_feature_message) against the separate kernels they replace (amx_sum_partials + count,
amx_mmd_fit, amx_mmd_reward / amx_mmd_reward_raw, amx_expert_cost): the same bits for w, w.w,
every reward / ipm / bonus and the expert cost, with and without a cost range, with and
without expert rows, for empty rollouts, and over repeated launches (the arrival counter
resets itself).  Reference: batch_reinforce.py:103-169, linear_cost.py:84-152."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def setup(n=9000, n_e=50000, F=512, seed=0):
    import amp_extensions_amd as amx
    from amp_extensions_amd import _native as N
    ctx = amx.AmxContext(197, 36, n_models=4, hidden=512, n_hidden=4, feat_dim=F, device=DEV)
    g = torch.Generator(device="cpu").manual_seed(seed)
    sc = float(np.sqrt(2.0 / F))
    phi = (torch.cos(torch.rand(n, F, generator=g) * 6.3) * sc).to(DEV)
    erows = (torch.cos(torch.rand(n_e, F, generator=g) * 6.3 + 0.3) * sc).to(DEV)
    phi_e = erows.double().mean(0).float()
    parts = (torch.randn((n + 127) // 128, F, generator=g, dtype=torch.float64) * 3.0).to(DEV)
    disc = (torch.rand(n, generator=g) * 0.2).to(DEV)
    return ctx, N, phi, erows, phi_e, parts, disc


def f32(n):
    return torch.empty(n, dtype=torch.float32, device=DEV)


@pytest.mark.parametrize("clamp,expert,n", [(1, True, 9000), (1, False, 9000), (0, False, 9000), (1, True, 0),
                                            (1, True, 5)])
def test_relabel_fused_matches_separate_kernels(clamp, expert, n):
    ctx, N, phi, erows, phi_e, parts, disc = setup()
    F, lib, h, s = 512, ctx.lib, ctx.h, ctx.stream
    lam, thr, cmin, cmax = 0.0025, 0.07, -1.0, 0.0
    n_parts = parts.shape[0]
    count = float(n if n else 1)
    # feature message vs sum_partials + count
    msg = torch.empty(F + 1, dtype=torch.float64, device=DEV)
    N.check(lib.amx_feature_message(h, parts.data_ptr(), n_parts, F, count, msg.data_ptr(), s), "msg")
    ref_sum = torch.empty(F, dtype=torch.float64, device=DEV)
    N.check(lib.amx_sum_partials(h, parts.data_ptr(), n_parts, F, ref_sum.data_ptr(), s), "sum")
    torch.cuda.synchronize()
    assert torch.equal(msg[:F], ref_sum) and msg[F].item() == count
    # separate kernels
    w0, m0 = f32(F), f32(1)
    N.check(lib.amx_mmd_fit(h, msg.data_ptr(), 0.0, phi_e.data_ptr(), F, w0.data_ptr(), m0.data_ptr(), s), "fit")
    r0, i0, b0 = f32(max(n, 1)), f32(max(n, 1)), f32(max(n, 1))
    if n:
        if clamp:
            N.check(lib.amx_mmd_reward(h, phi.data_ptr(), F, w0.data_ptr(), F, disc.data_ptr(), thr, lam, cmin, cmax,
                                       r0.data_ptr(), i0.data_ptr(), b0.data_ptr(), n, s), "reward")
        else:
            N.check(lib.amx_mmd_reward_raw(h, phi.data_ptr(), F, w0.data_ptr(), F, disc.data_ptr(), lam,
                                           r0.data_ptr(), i0.data_ptr(), b0.data_ptr(), n, s), "reward_raw")
    eo0 = torch.empty(1025, dtype=torch.float64, device=DEV)
    em0 = f32(1)
    if expert:
        N.check(lib.amx_expert_cost(h, erows.data_ptr(), F, w0.data_ptr(), F, erows.shape[0], cmin, cmax,
                                    eo0.data_ptr(), em0.data_ptr(), lam, s), "expert")
    # fused, three times (counter reset)
    counter = torch.zeros(4, dtype=torch.int32, device=DEV)
    for _ in range(3):
        w1, m1 = f32(F), f32(1)
        r1, i1, b1 = f32(max(n, 1)), f32(max(n, 1)), f32(max(n, 1))
        eo1 = torch.zeros(1025, dtype=torch.float64, device=DEV)
        em1 = f32(1)
        N.check(lib.amx_mmd_relabel(h, msg.data_ptr(), 0.0, phi_e.data_ptr(), F, w1.data_ptr(), m1.data_ptr(),
                                    phi.data_ptr(), F, disc.data_ptr(), thr, lam, clamp, cmin, cmax, r1.data_ptr(),
                                    i1.data_ptr(), b1.data_ptr(), n, erows.data_ptr() if expert else None, F,
                                    erows.shape[0], eo1.data_ptr(), em1.data_ptr(), counter.data_ptr(), s),
                "relabel")
        torch.cuda.synchronize()
        assert torch.equal(w0, w1) and torch.equal(m0, m1)
        if n:
            assert torch.equal(r0[:n], r1[:n]) and torch.equal(i0[:n], i1[:n]) and torch.equal(b0[:n], b1[:n])
        if expert:
            assert torch.equal(eo0[0], eo1[0]) and torch.equal(em0, em1)
        assert int(counter[0].item()) == 0


def test_relabel_fused_rejects_bad_arguments():
    ctx, N, phi, erows, phi_e, parts, disc = setup(n=256, n_e=512)
    lib, h, s = ctx.lib, ctx.h, ctx.stream
    msg = torch.zeros(513, dtype=torch.float64, device=DEV)
    w, m = f32(512), f32(1)
    # expert cost without a cost range
    rc = lib.amx_mmd_relabel(h, msg.data_ptr(), 1.0, phi_e.data_ptr(), 512, w.data_ptr(), m.data_ptr(), None, 512,
                             None, 1.0, 0.1, 0, 0.0, 0.0, None, None, None, 0, erows.data_ptr(), 512, 512,
                             None, None, None, s)
    assert rc != 0 and b"expert" in lib.amx_last_error()
    rc = lib.amx_mmd_relabel(h, msg.data_ptr(), 1.0, phi_e.data_ptr(), 500, w.data_ptr(), m.data_ptr(), None, 512,
                             None, 1.0, 0.1, 1, -1.0, 0.0, None, None, None, 0, None, 512, 0, None, None, None, s)
    assert rc != 0
