"""The device policy kernel (amx_policy_act: three v_mfma_f32_16x16x4_f32 layers over the 16
lanes of a workgroup, one Box-Muller per action pair) at shapes away from the bench's: state
and hidden widths that are not multiples of 4 or 16 (the zero-padded chunks and the unit
blocks past H), odd action counts (the last pair's single normal), hidden widths of one to six 16-unit blocks
(four, two or one K part per block), lane counts that leave a partial workgroup; a width whose
weights do not fit the workgroup's LDS staging is rejected by the ABI check.  Means against
the oracle's FCNetwork (gaussian_mlp.py / fc_network.py:42-55, rel 1e-4 + abs 1e-6), noise
against the oracle's Philox + Box-Muller (1e-12), injected noise and eval mode exact given the
device mean.  Reference: mjrl/mjrl/policies/gaussian_mlp.py:95-104."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("S,A,hidden,B", [(197, 36, (32, 32), 1000), (50, 7, (20, 24), 37), (226, 28, (64, 64), 300),
                                          (13, 3, (5, 17), 16), (100, 36, (96, 64), 65), (41, 64, (16, 48), 129), (20, 65, (8, 8), 5)])
def test_policy_shapes_match_oracle(S, A, hidden, B):
    import amp_extensions_amd as amx
    ctx = amx.AmxContext(S, A, n_models=1, hidden=16, n_hidden=1, feat_dim=256, device=DEV)
    pw, log_std = R.init_policy_weights(S, A, hidden, seed=100 + S, init_log_std=-0.25)
    # lift the output layer off its 1e-2 init so the means test the whole MLP at scale
    pw[-1] = (pw[-1][0] * 50.0, pw[-1][1] * 50.0)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=77)
    rs = np.random.RandomState(S + A)
    ob = rs.randn(B, S)
    d_ob = torch.from_numpy(ob).to(DEV)
    act = torch.empty(B, A, dtype=torch.float64, device=DEV)
    mean = torch.empty(B, A, dtype=torch.float32, device=DEV)
    ref_mean = np.stack([R.policy_mean(pw, ob[b]) for b in range(B)])
    scale = np.exp(np.float64(log_std.numpy()))
    # Philox noise
    pol.act(d_ob, B, act, counter=11, mean_out=mean)
    m = mean.cpu().numpy()
    np.testing.assert_allclose(m, ref_mean, rtol=1e-4, atol=1e-6)
    z = R.policy_noise(77, 11, B, A)
    np.testing.assert_allclose(act.cpu().numpy() - m.astype(np.float64), scale * z, rtol=1e-12, atol=1e-12)
    # injected noise: the fp64 action algebra is exact given the device mean
    noise = torch.from_numpy(rs.randn(B, A)).to(DEV)
    pol.act(d_ob, B, act, counter=11, noise=noise, mean_out=mean)
    np.testing.assert_array_equal(act.cpu().numpy(), m.astype(np.float64) + scale * noise.cpu().numpy())
    # eval mode: the mean itself
    pol.act(d_ob, B, act, counter=11, eval_mode=True, mean_out=mean)
    np.testing.assert_array_equal(act.cpu().numpy(), m.astype(np.float64))


def test_policy_rejects_oversized_shapes():
    import amp_extensions_amd as amx
    from amp_extensions_amd._native import AmxNativeError
    S, A = 197, 36  # W1 256 x 197 + W2 256 x 256 do not fit the 160 KB of LDS
    ctx = amx.AmxContext(S, A, n_models=1, hidden=16, n_hidden=1, feat_dim=256, device=DEV)
    pw, log_std = R.init_policy_weights(S, A, (256, 256), seed=1)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
    ob = torch.zeros(4, S, dtype=torch.float64, device=DEV)
    act = torch.empty(4, A, dtype=torch.float64, device=DEV)
    with pytest.raises(AmxNativeError, match="LDS"):
        pol.act(ob, 4, act, counter=0)
