"""Device NPG policy update: the learner step that consumes the rollout
(mjrl NPG.train_from_paths, mjrl/mjrl/algos/npg_cg.py:113-199), next to the rollout engine.

The per-sample work (policy forward, Jacobian-vector products, back-propagation and the
reduction of per-sample gradients) is the HIP kernel `amx_npg_pass` (csrc/amx_npg.hip); the
10-iteration conjugate gradient (mjrl/mjrl/utils/cg_solve.py) is fp64 vector algebra on the
device between passes.  Parameters live in the reference's flat order (MLP.trainable_params:
W1, b1, W2, b2, W3, b3, log_std — gaussian_mlp.py:44-62), so `get_param_values` /
`set_param_values` exchange the same vectors as the reference policy.

Same semantics as the reference with hvp_sample_frac = 1 (MILO's default,
milo/milo/arguments.py:122) and no input normalization (FCNetwork's default in_shift/in_scale:
(x - 0) / (1 + 1e-8) == x in float32); a subsampled FIM or input normalization raise.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _native as N
from .engine import AmxContext

NPG_VPG, NPG_FVP, NPG_EVAL = 0, 1, 2


def pack_policy(layers, log_std) -> np.ndarray:
    """[(W1, b1), (W2, b2), (W3, b3)], log_std -> the reference's flat fp32 parameter vector."""
    parts = []
    for W, b in layers:
        parts += [np.asarray(torch.as_tensor(W).detach().cpu().float()).ravel(),
                  np.asarray(torch.as_tensor(b).detach().cpu().float()).ravel()]
    parts.append(np.asarray(torch.as_tensor(log_std).detach().cpu().float()).ravel())
    return np.concatenate(parts).astype(np.float32)


def unpack_policy(flat, S: int, A: int, hidden=(32, 32)):
    """Inverse of pack_policy: ([(W, b)] * 3, log_std) as CPU float32 tensors."""
    flat = np.asarray(flat, dtype=np.float32)
    sizes = (S,) + tuple(hidden) + (A,)
    layers, i = [], 0
    for k in range(len(sizes) - 1):
        o, n = sizes[k + 1], sizes[k]
        W = torch.from_numpy(flat[i:i + o * n].reshape(o, n).copy())
        i += o * n
        b = torch.from_numpy(flat[i:i + o].copy())
        i += o
        layers.append((W, b))
    return layers, torch.from_numpy(flat[i:i + A].copy())


class DeviceNPG:
    """NPG (npg_cg.py:26-199) for the mjrl Gaussian MLP policy, on the device.

    `policy_layers`/`log_std`: the current policy (nn.Linear layout).  `policy` (optional): a
    DevicePolicy to refresh after every update (the rollout's sampler)."""

    def __init__(self, ctx: AmxContext, policy_layers, log_std, normalized_step_size=0.01, const_learn_rate=None,
                 FIM_invert_args=None, hvp_sample_frac=1.0, kl_dist=None, min_log_std=-3.0,
                 input_normalization=None, policy=None, residual_tol=1e-10):
        if hvp_sample_frac is not None and hvp_sample_frac < 0.99:
            raise NotImplementedError("subsampled Fisher (hvp_sample_frac < 1) is not implemented")
        if input_normalization:
            raise NotImplementedError("running input normalization is not implemented")
        if len(policy_layers) != 3 or any(W.shape[0] != 32 for W, _ in policy_layers[:2]):
            raise NotImplementedError("the device NPG kernel supports the (32, 32) tanh MLP (MILO's actor)")
        self.ctx = ctx
        self.S, self.A = ctx.S, ctx.A
        if policy_layers[0][0].shape[1] != self.S or policy_layers[2][0].shape[0] != self.A:
            raise ValueError("policy shapes do not match the context's S, A")
        FIM_invert_args = FIM_invert_args or {"iters": 10, "damping": 1e-4}
        self.cg_iters = int(FIM_invert_args["iters"])
        self.cg_fold = True  # the CG vector step folded into the next Fisher-vector pass
        self.damping = float(FIM_invert_args["damping"])
        self.alpha = const_learn_rate
        self.n_step_size = normalized_step_size if kl_dist is None else 2.0 * kl_dist
        self.min_log_std = float(min_log_std)
        self.residual_tol = residual_tol
        self.policy = policy
        self.P = int(ctx.lib.amx_npg_param_count(self.S, self.A))
        self.theta = torch.from_numpy(pack_policy(policy_layers, log_std)).to(ctx.device)
        assert self.theta.numel() == self.P
        self._bufs = {}

    # ---- parameters (reference flat order) ----------------------------------------------
    def get_param_values(self) -> np.ndarray:
        return self.theta.cpu().numpy().copy()

    def set_param_values(self, new_params) -> None:
        """MLP.set_param_values (gaussian_mlp.py:71-94): float32, log_std clamped at min_log_std.
        A device tensor stays on the device (no host round trip)."""
        if isinstance(new_params, torch.Tensor):
            t = new_params.detach().to(self.ctx.device, torch.float32).clone()
        else:
            t = torch.as_tensor(np.asarray(new_params), dtype=torch.float32).to(self.ctx.device).clone()
        t[-self.A:] = torch.clamp(t[-self.A:], min=self.min_log_std)
        self.theta = t.contiguous()
        if self.policy is not None:
            self.policy.sync_from(*self._layers_view())

    def _layers_view(self):
        """([(W, b)] * 3, log_std) as device views of theta (reference flat order)."""
        sizes = (self.S, 32, 32, self.A)
        layers, i = [], 0
        for k in range(3):
            o, n = sizes[k + 1], sizes[k]
            W = self.theta[i:i + o * n].view(o, n)
            i += o * n
            layers.append((W, self.theta[i:i + o]))
            i += o
        return layers, self.theta[i:i + self.A]

    # ---- passes --------------------------------------------------------------------------
    def _rows_per_block(self, n: int) -> int:
        # one block per CU (the pass kernel holds ~140 KB of LDS): one wave of blocks
        return max(32, int(math.ceil(n / 256 / 32)) * 32)

    def _pass(self, mode, obs, act, adv, vec, gate=None, hcache=None, reduce=True, out=None):
        """One pass (amx_npg_pass_ex) and its block-order reduction (into `out` when given);
        reduce=False returns the [blocks][width] partials instead (the CG folds their reduction
        into its step)."""
        c = self.ctx
        n = obs.shape[0]
        rpb = self._rows_per_block(n)
        nb = (n + rpb - 1) // rpb
        width = 2 if mode == NPG_EVAL else self.P
        key = (nb, width)
        part = self._bufs.get(key)
        if part is None:
            part = self._bufs[key] = torch.empty(nb, width, dtype=torch.float64, device=c.device)
        od = N.AMX_IN_F64 if obs.dtype == torch.float64 else N.AMX_IN_F32
        ad = N.AMX_IN_F64 if act.dtype == torch.float64 else N.AMX_IN_F32
        g = None if gate is None else gate.data_ptr()
        N.check(c.lib.amx_npg_pass_ex(c.h, mode, n, obs.data_ptr(), od, obs.stride(0), act.data_ptr(), ad,
                                      act.stride(0), None if adv is None else adv.data_ptr(),
                                      self.theta.data_ptr(), None if vec is None else vec.data_ptr(), rpb,
                                      part.data_ptr(), g, None if hcache is None else hcache.data_ptr(), c.stream),
                "amx_npg_pass")
        if not reduce:
            return part
        if out is None:
            out = torch.empty(width, dtype=torch.float64, device=c.device)
        N.check(c.lib.amx_npg_reduce_gated(c.h, part.data_ptr(), nb, width, out.data_ptr(), g, c.stream),
                "amx_npg_reduce")
        return out

    def _inputs(self, observations, actions, advantages=None):
        dev = self.ctx.device
        obs = torch.as_tensor(observations).to(dev)
        act = torch.as_tensor(actions).to(dev)
        # the policy reads float32(obs) / float32(act) (gaussian_mlp.py:112-117): one cast here
        # serves every pass of the update and lets the pass kernel take 64-row chunks
        obs = obs.to(torch.float32).contiguous()
        act = act.to(torch.float32).contiguous()
        if obs.dim() != 2 or obs.shape[1] != self.S or act.shape != (obs.shape[0], self.A):
            raise ValueError(f"observations {tuple(obs.shape)} / actions {tuple(act.shape)} do not match S, A")
        adv = None
        if advantages is not None:
            adv = torch.as_tensor(advantages).to(dev, torch.float64).contiguous()
            if adv.numel() != obs.shape[0]:
                raise ValueError("advantages must have one entry per observation")
        return obs, act, adv

    def flat_vpg(self, observations, actions, advantages) -> torch.Tensor:
        """BatchREINFORCE.flat_vpg (batch_reinforce.py:58-62) at new == old: fp64 [P]."""
        obs, act, adv = self._inputs(observations, actions, advantages)
        return self._pass(NPG_VPG, obs, act, adv, None)

    def _ls_curvature(self) -> torch.Tensor:
        """d^2 mean_kl / d log_std^2 at new == old (gaussian_mlp.py:144-155 with Dr's 1e-8):
        (8 s^2 - 4 s eps) / (2 s + eps)^2, s = exp(log_std)^2 -- one launch (amx_npg_curvature)."""
        c = self.ctx
        curv = torch.empty(self.A, dtype=torch.float64, device=c.device)
        N.check(c.lib.amx_npg_curvature(c.h, self.theta.data_ptr(), self.P, self.A, curv.data_ptr(), c.stream),
                "amx_npg_curvature")
        return curv

    def HVP(self, observations, actions, vector, regu_coef=None) -> torch.Tensor:
        """NPG.HVP (npg_cg.py:87-106): Fisher (mean_kl Hessian) times `vector` + damping."""
        obs, act, _ = self._inputs(observations, actions)
        return self._hvp(obs, act, torch.as_tensor(vector).to(self.ctx.device), regu_coef)

    def _hvp(self, obs, act, v, regu_coef=None):
        regu = self.damping if regu_coef is None else regu_coef
        v32 = v.to(torch.float32).contiguous()   # the reference casts the vector to float32
        h = self._pass(NPG_FVP, obs, act, None, v32)
        h[-self.A:] += self._ls_curvature() * v32[-self.A:].double()
        return h + regu * v.to(torch.float64)  # hvp_flat + regu_coef * vector (npg_cg.py:105: the fp64 vector)

    def _hcache(self, n: int) -> torch.Tensor:
        """The per-sample theta forward (H1 | H2, [n][64] fp32) the VPG pass writes and the CG's
        Fisher-vector passes read (amx_npg_pass_ex), grown on demand."""
        hc = self._bufs.get("hcache")
        if hc is None or hc.shape[0] < n:
            hc = self._bufs["hcache"] = torch.empty(n, 64, dtype=torch.float32, device=self.ctx.device)
        return hc

    def cg_solve(self, obs, act, b: torch.Tensor, hcache=None) -> torch.Tensor:
        """mjrl/mjrl/utils/cg_solve.py:3-23 (starts from zeros; stops at rdotr < tol) with
        NPG.HVP as the operator.  Each iteration is one Fisher-vector pass and one column-sum
        launch (amx_npg_cg_reduce: z and the p.z parts per block); the vector step (x, r, p from
        fixed-order block parts) runs at the head of the NEXT iteration's pass (amx_npg_pass_cg,
        the same bits as the step's own launch) and once more, alone, after the last
        (amx_npg_cg_xrp).  `cg_fold = False` runs the round-5 form instead: the pass on p32, then
        amx_npg_cg_tail (the reduction and the step in two launches).  The early stop is the
        device-side `live` flag (a finished solve leaves x unchanged), so no host sync between
        iterations; after the stop the passes and reductions are empty launches.  `hcache`: the
        theta forward written by this update's VPG pass (train_from_arrays), so every product
        skips layers 1-2 at theta (bit-identical products)."""
        c = self.ctx
        P = self.P
        dev = c.device
        b = b.to(torch.float64).contiguous()
        x, r, p, r2, p2 = (torch.empty(P, dtype=torch.float64, device=dev) for _ in range(5))
        p32, p32b = (torch.empty(P, dtype=torch.float32, device=dev) for _ in range(2))
        state, state2 = (torch.empty(2, dtype=torch.float64, device=dev) for _ in range(2))
        curv = torch.empty(self.A, dtype=torch.float64, device=dev)  # the log_std curvature, same launch
        N.check(c.lib.amx_npg_cg_init_ls(c.h, P, self.A, self.theta.data_ptr(), curv.data_ptr(), b.data_ptr(),
                                         x.data_ptr(), r.data_ptr(), p.data_ptr(), p32.data_ptr(), state.data_ptr(),
                                         c.stream), "amx_npg_cg_init_ls")
        work = self._bufs.get("cg_work")
        if work is None:
            work = self._bufs["cg_work"] = torch.empty(int(c.lib.amx_npg_cg_tail_work(P)), dtype=torch.float64,
                                                       device=dev)
        hc = hcache if obs.dtype == torch.float32 else None
        if not self.cg_fold:
            for _ in range(self.cg_iters):
                part = self._pass(NPG_FVP, obs, act, None, p32, gate=state, hcache=hc, reduce=False)
                # the partials' column sums and the vector step (amx_npg_cg_tail: two launches); r
                # and the state alternate buffers from one iteration to the next
                N.check(c.lib.amx_npg_cg_tail(c.h, part.data_ptr(), part.shape[0], P, self.A, curv.data_ptr(),
                                              self.damping, self.residual_tol, x.data_ptr(), r.data_ptr(),
                                              r2.data_ptr(), p.data_ptr(), p32.data_ptr(), state.data_ptr(),
                                              state2.data_ptr(), work.data_ptr(), c.stream), "amx_npg_cg_tail")
                r, r2 = r2, r
                state, state2 = state2, state
            return x
        n = obs.shape[0]
        rpb = self._rows_per_block(n)
        od = N.AMX_IN_F64 if obs.dtype == torch.float64 else N.AMX_IN_F32
        for it in range(self.cg_iters):
            if it == 0:
                part = self._pass(NPG_FVP, obs, act, None, p32, gate=state, hcache=hc, reduce=False)
            else:
                # the previous iteration's vector step, then the product with its p'; r, p, p32
                # and the state alternate buffers (every block reads all of them)
                N.check(c.lib.amx_npg_pass_cg(c.h, n, obs.data_ptr(), od, obs.stride(0), self.theta.data_ptr(), rpb,
                                              part.data_ptr(), None if hc is None else hc.data_ptr(),
                                              self.residual_tol, x.data_ptr(), r.data_ptr(), r2.data_ptr(),
                                              p.data_ptr(), p2.data_ptr(), p32b.data_ptr(), state.data_ptr(),
                                              state2.data_ptr(), work.data_ptr(), c.stream), "amx_npg_pass_cg")
                r, r2, p, p2, p32, p32b, state, state2 = r2, r, p2, p, p32b, p32, state2, state
            N.check(c.lib.amx_npg_cg_reduce(c.h, part.data_ptr(), part.shape[0], P, self.A, curv.data_ptr(),
                                            self.damping, p.data_ptr(), p32.data_ptr(), state.data_ptr(),
                                            work.data_ptr(), c.stream), "amx_npg_cg_reduce")
        if self.cg_iters > 0:
            N.check(c.lib.amx_npg_cg_xrp(c.h, P, self.residual_tol, x.data_ptr(), r.data_ptr(), r2.data_ptr(),
                                         p.data_ptr(), p32.data_ptr(), state.data_ptr(), state2.data_ptr(),
                                         work.data_ptr(), c.stream), "amx_npg_cg_xrp")
        return x

    def surrogate_kl(self, obs, act, adv_w, new_theta) -> tuple[float, float]:
        """(CPI_surrogate, kl_old_new) of new_theta against the current parameters."""
        tot = self._pass(NPG_EVAL, obs, act, adv_w, new_theta.to(torch.float32).contiguous())
        n = obs.shape[0]
        return float(tot[0]) / n, float(tot[1]) / n

    # ---- the update ------------------------------------------------------------------------
    def train_from_arrays(self, observations, actions, advantages, whiten: bool = True) -> dict:
        """NPG.train_from_paths on concatenated arrays (npg_cg.py:113-199): whitening
        (batch_reinforce.py:284-285), VPG, CG, step size, update with the log_std clamp,
        surr_after and kl_dist.  Returns the reference's infos entries."""
        obs, act, adv = self._inputs(observations, actions, advantages)
        c = self.ctx
        n = obs.shape[0]
        if whiten:  # (adv - mean) / (std + 1e-6), population std: amx_adv_whiten (per-block parts, then combine + apply)
            w = torch.empty_like(adv)
            stats = torch.empty(2, dtype=torch.float64, device=c.device)
            N.check(c.lib.amx_adv_whiten(c.h, 1, n, None, None, n, adv.data_ptr(), 1e-6, w.data_ptr(),
                                         stats.data_ptr(), c.stream), "amx_adv_whiten")
            adv = w
        hc = self._hcache(n)
        vpg = self._pass(NPG_VPG, obs, act, adv, None, hcache=hc)
        npg = self.cg_solve(obs, act, vpg, hcache=hc)
        # gdot, the step size and the clamped new parameters in one launch (amx_npg_apply_step)
        new = torch.empty(self.P, dtype=torch.float32, device=c.device)
        # [alpha, n_step_size, gdot | surr, kl]: the step kernel and the eval reduction write the
        # two ends of one buffer, read back in one copy (no concatenation kernel)
        res = torch.empty(5, dtype=torch.float64, device=c.device)
        scal = res[:3]
        use_alpha = self.alpha is not None
        N.check(c.lib.amx_npg_apply_step(c.h, self.P, self.A, vpg.data_ptr(), npg.data_ptr(), self.theta.data_ptr(),
                                         int(use_alpha), float(self.alpha) if use_alpha else 0.0,
                                         float(self.n_step_size), self.min_log_std, new.data_ptr(),
                                         scal.data_ptr(), c.stream), "amx_npg_apply_step")
        self._pass(NPG_EVAL, obs, act, adv, new, out=res[3:])
        self.theta = new  # already float32 with the log_std clamp (set_param_values' form)
        if self.policy is not None:
            self.policy.sync_from(*self._layers_view())
        # the update's one host sync: the reference's infos are python floats
        alpha_h, delta_h, _, surr_h, kl_h = res.tolist()
        return {"vpg_grad": vpg, "npg_grad": npg, "alpha": alpha_h, "delta": delta_h, "surr_before": 0.0,
                "surr_after": surr_h / n, "kl_dist": kl_h / n, "advantages": adv}

    def train_from_paths(self, paths, infos: dict | None = None):
        """Reference surface: mjrl path dicts (observations, actions, advantages, rewards) ->
        base_stats [mean, std, min, max] of path returns; infos updated as the reference's."""
        obs = np.concatenate([p["observations"] for p in paths])
        act = np.concatenate([p["actions"] for p in paths])
        adv = np.concatenate([p["advantages"] for p in paths])
        out = self.train_from_arrays(obs, act, adv)
        if infos is not None:
            infos.update({k: v for k, v in out.items()})
        returns = [float(np.sum(p["rewards"])) for p in paths]
        return [float(np.mean(returns)), float(np.std(returns)), float(np.min(returns)), float(np.max(returns))]

    def train_from_engine(self, engine, advantages: torch.Tensor) -> dict:
        """Update from the rollout engine's buffers without a host round trip: the recorded
        transitions obs[:T], acts[:T] ([T, B] rows) and GAE advantages [T, B]."""
        T, B = engine.t, engine.B
        obs = engine.obs[:T].reshape(T * B, self.S)
        act = engine.acts[:T].reshape(T * B, self.A)
        return self.train_from_arrays(obs, act, advantages.reshape(T * B))
