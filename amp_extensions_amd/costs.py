"""Device-backed drop-ins for the reference cost objects.

* `RBFLinearCost` — milo/milo/linear_cost.py:6-152 (MILO RFF MMD cost + pessimism bonus)
* `GAILCost`      — milo/milo/gail_cost.py:44-279, inference surface (AMP least-squares
                    discriminator reward + bonus); discriminator training is out of scope.

Initialisation reproduces the reference's torch-CPU RNG stream exactly (seed, bandwidth
draw, nn.Linear construction order), so the same seed yields the same W, b, bandwidth and
discriminator weights; every per-sample computation then runs in the HIP kernels with the
expert features resident in HBM.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from .engine import AmxContext, RffMap, round_up, split_bf16x3, split_f16x2


def device_discrepancy(ensemble, states, actions) -> torch.Tensor:
    """get_action_discrepancy (dynamics.py:154-165) left on the GPU, for any ensemble the
    surfaces accept (this package's DynamicsEnsemble / DeviceEnsemble, or the reference's own
    object, converted once: ensemble.as_device_ensemble)."""
    from .ensemble import as_device_ensemble
    return as_device_ensemble(ensemble).get_action_discrepancy(states, actions)

# cost-input row of a transition (linear_cost.py:115-127, gail_cost.py:258-268); "amp" is
# the AMP observation of (s, s') (SceneImitateAMP::BuildAMPObs, via a ReferenceMotion)
INPUT_TYPES = ("ss", "sa", "sas", "s", "amp")


def input_width(input_type: str, S: int, A: int, motion=None) -> int:
    """Width of the cost-input row of `input_type` for state size S and action size A."""
    if input_type == "amp":
        if motion is None:
            raise ValueError("input_type 'amp' needs the ReferenceMotion (motion=...)")
        return motion.amp_obs_size
    return {"ss": 2 * S, "sa": S + A, "sas": 2 * S + A, "s": S}[input_type]


def cost_input(input_type: str, states, actions, next_states, motion=None) -> torch.Tensor:
    """float32 cost-input rows [n, width] of `input_type` (the reference's torch.cat branches)."""
    if input_type == "sa":
        return torch.cat([states.float(), actions.float()], dim=1)
    if input_type == "ss":
        assert next_states is not None
        return torch.cat([states.float(), next_states.float()], dim=1)
    if input_type == "sas":
        return torch.cat([states.float(), actions.float(), next_states.float()], dim=1)
    if input_type == "s":
        return states.float()
    if input_type == "amp":
        assert next_states is not None and motion is not None
        return motion.amp_obs_from_states(states.double().contiguous(), next_states.double().contiguous()).float()
    raise NotImplementedError("Input type not implemented")


def _check_input_type(input_type: str, motion) -> None:
    if input_type not in INPUT_TYPES:
        raise NotImplementedError("Input type not implemented")
    if input_type == "amp" and motion is None:
        raise ValueError("input_type 'amp' needs the ReferenceMotion (motion=...)")


class RBFLinearCost:
    """MMD cost with random-Fourier-feature representations (linear_cost.py:6-152).

    Same constructor arguments and methods as the reference; tensors returned by the
    cost methods live on the engine's device.
    """

    def __init__(self, expert_data: torch.Tensor, feature_dim=1024, input_type="ss", cost_range=(-1.0, 0.0),
                 bw_quantile=0.1, bw_samples=100000, lambda_b=1.0, lr=0.0, seed=100, ctx: AmxContext | None = None,
                 device="cuda", gemm: str = "f16x3", motion=None):
        """`gemm` selects the feature GEMM: "f16x3" (scaled 2-limb fp16 split) or "bf16x6"
        (3-limb bf16 split), both fp32-level error, or "f32" (f32 MFMA); `motion` (a
        ReferenceMotion) is needed for input_type "amp" (expert
        rows = AMP observations); everything else follows the reference constructor."""
        _check_input_type(input_type, motion)
        torch.manual_seed(seed)          # linear_cost.py:34-35
        np.random.seed(seed)
        expert_cpu = expert_data.detach().float().cpu()
        input_dim = expert_cpu.size(1)
        self.input_type = input_type
        self.input_dim = input_dim
        self.motion = motion
        self.feature_dim = feature_dim
        self.cost_range = cost_range
        if cost_range is not None:
            self.c_min, self.c_max = float(cost_range[0]), float(cost_range[1])
        self.lambda_b = float(lambda_b)
        self.lr = lr
        self.quantile = bw_quantile
        self.bw_samples = bw_samples
        self.bw = self.fit_bandwidth(expert_cpu)                  # :50 (torch-CPU RNG order)
        rff = nn.Linear(input_dim, feature_dim)                   # :53
        rff.bias.data = (torch.rand_like(rff.bias.data) - 0.5) * 2.0 * np.pi          # :54
        rff.weight.data = torch.rand_like(rff.weight.data) / (self.bw + 1e-8)          # :55
        self.rff_weight, self.rff_bias = rff.weight.data, rff.bias.data
        if ctx is None:
            S = input_dim // 2 if input_type == "ss" else input_dim
            ctx = AmxContext(S, 1, n_models=1, hidden=128, n_hidden=0, feat_dim=feature_dim, device=device)
        self.ctx = ctx
        self.map = RffMap(ctx, self.rff_weight, self.rff_bias, gemm=gemm)
        self.w = None
        # expert features resident in HBM (:61-62); phi_e from fp64 column sums
        phi, tot = self.map.embed(expert_cpu)
        self.expert_rep = phi
        self.n_expert = expert_cpu.shape[0]
        self.phi_e = (tot / self.n_expert).float()
        self._expert_out = torch.empty(1 + 1024, dtype=torch.float64, device=ctx.device)
        self._expert_mean = None  # fp32 [1]: get_expert_cost's result (amx_expert_cost mean_out)
        # set when the last relabel_device launch also computed the expert cost for the current w
        self._expert_fresh = False
        self._counter = torch.zeros(4, dtype=torch.int32, device=ctx.device)  # amx_mmd_relabel's arrivals
        # expert rows this rank scores (shard_expert: a contiguous block per rank, partial sums
        # all-reduced asynchronously -- the expert cost only feeds the bonus_mmd log)
        self._elo, self._ehi = 0, self.n_expert
        self._ear = None   # allreduce_async of the sharded partial sum (None: one rank, whole buffer)
        self._eh = None    # the pending all-reduce handle of the last sharded partial sum
        self._estate = "global"  # sharded sum in _expert_out[0]: "partial" (this rank's) or "global"
        self._escale = torch.tensor([1.0 - lambda_b], dtype=torch.float32, device=ctx.device)

    # linear_cost.py:73-82
    def fit_bandwidth(self, data: torch.Tensor) -> float:
        n = data.shape[0]
        i0 = torch.randint(low=0, high=n, size=(self.bw_samples,))
        i1 = torch.randint(low=0, high=n, size=(self.bw_samples,))
        norm = torch.norm(data[i0, :] - data[i1, :], dim=1)
        return torch.quantile(norm, q=self.quantile).item()

    def get_rep(self, x: torch.Tensor) -> torch.Tensor:
        """linear_cost.py:64-71."""
        return self.map.embed(x)[0]

    def fit_w_device(self, phi_sum: torch.Tensor, count: float) -> torch.Tensor:
        """Closed-form witness from an (already all-reduced) fp64 feature sum; returns w.w as
        a 1-element device tensor (no host synchronisation)."""
        c = self.ctx
        self._alloc_w()
        self._expert_fresh = False
        N.check(c.lib.amx_mmd_fit(c.h, phi_sum.data_ptr(), float(count), self.phi_e.data_ptr(), self.feature_dim,
                                  self.w.data_ptr(), self._mmd.data_ptr(), c.stream), "amx_mmd_fit")
        return self._mmd

    def _alloc_w(self) -> None:
        if self.w is None:
            c = self.ctx
            self.w = torch.empty(self.feature_dim, dtype=torch.float32, device=c.device)
            self._mmd = torch.empty(1, dtype=torch.float32, device=c.device)

    def shard_expert(self, rank: int, world: int, allreduce_async) -> None:
        """Score only this rank's contiguous block of the resident expert rows in the relabel
        and sum the ranks' fp64 partial sums with `allreduce_async(buf)` (returns a handle with
        .wait(), e.g. dist.all_reduce(async_op=True)), issued by expert_allreduce() off the
        rollout's critical path: get_expert_cost (linear_cost.py:105-109; bonus_mmd's expert
        term, batch_reinforce.py:169, a log value) waits for it when read.  SURVEY §8(e): phi_e
        replicated, the expert buffer's cost sharded, one scalar all-reduce for the log."""
        from .dist import shard
        if world > self.n_expert:
            raise ValueError(f"{self.n_expert} expert rows cannot be sharded over {world} ranks")
        self._elo, self._ehi = shard(self.n_expert, rank, world)
        self._ear = allreduce_async if world > 1 else None

    @property
    def expert_sharded(self) -> bool:
        return self._ear is not None

    def expert_allreduce(self):
        """Issue the all-reduce of the last relabel's partial expert sum (sharded mode, once per
        partial sum; no-op otherwise); returns the handle (the next relabel waits for it,
        GPU-side, before it overwrites the sum)."""
        if self._ear is None or not self._expert_fresh or self._estate != "partial":
            return None
        self._eh = self._ear(self._expert_out[:1])
        self._estate = "global"
        return self._eh

    def expert_allreduce_replayed(self):
        """expert_allreduce after a replayed graph whose relabel wrote a new partial sum (the
        graph's `after` hook: the captured launch does not pass through relabel_device)."""
        if self._ear is None or self.cost_range is None:
            return None
        self._expert_fresh, self._estate = True, "partial"
        return self.expert_allreduce()

    def wait_expert_allreduce(self) -> None:
        """Queue the wait (GPU-side) for the pending expert-sum all-reduce (graph replays call it
        before the graph whose relabel overwrites the sum; eager relabels call it themselves)."""
        if self._eh is not None and not torch.cuda.is_current_stream_capturing():
            self._eh.wait()
            self._eh = None

    def _expert_args(self):
        """(rows pointer, row count, mean_out) of the expert rows this rank scores."""
        ld = self.expert_rep.stride(0)
        ptr = self.expert_rep.data_ptr() + self._elo * ld * self.expert_rep.element_size()
        mean = None if self._ear is not None else self._expert_mean.data_ptr()
        return ptr, self._ehi - self._elo, mean

    def relabel_device(self, msg: torch.Tensor, phi, ldphi: int, disc, thr: float, reward, ipm, wb,
                       n: int) -> torch.Tensor:
        """The relabel tail in one launch (amx_mmd_relabel): w and w.w from the (all-reduced)
        [sum phi | count] message, the rewards of n rollout rows (raw device pointers), and,
        with a cost range, the expert cost for the new w (get_expert_cost then returns it
        without another pass).  Returns w.w (device, no host synchronisation)."""
        c = self.ctx
        self._alloc_w()
        expert = self.cost_range is not None
        if expert and self._expert_mean is None:
            self._expert_mean = torch.empty(1, dtype=torch.float32, device=c.device)
        self.wait_expert_allreduce()  # the previous partial sum's all-reduce reads the buffer this launch writes
        eptr, ne, emean = self._expert_args() if expert else (None, self.n_expert, None)
        N.check(c.lib.amx_mmd_relabel(c.h, msg.data_ptr(), 0.0, self.phi_e.data_ptr(), self.feature_dim,
                                      self.w.data_ptr(), self._mmd.data_ptr(), phi, ldphi, disc, float(thr),
                                      self.lambda_b, 1 if expert else 0, self.c_min if expert else 0.0,
                                      self.c_max if expert else 0.0, reward, ipm, wb, n,
                                      eptr, self.expert_rep.stride(0), ne, self._expert_out.data_ptr(),
                                      emean, self._counter.data_ptr(), c.stream), "amx_mmd_relabel")
        self._expert_fresh = expert
        if expert and self._ear is not None and not torch.cuda.is_current_stream_capturing():
            # (a captured launch: expert_allreduce_replayed after each replay).  The partial sum's
            # all-reduce is issued here, right behind the relabel, so every rank issues the same
            # collective sequence whether or not it later reads get_expert_cost (which only waits)
            self._estate = "partial"
            self.expert_allreduce()
        return self._mmd

    def fit_w(self, phi_sum: torch.Tensor, count: float) -> float:
        """fit_w_device + the reference's Python-float return (linear_cost.py:94)."""
        return float(self.fit_w_device(phi_sum, count).item())

    def fit_cost(self, data_pi: torch.Tensor) -> float:
        """linear_cost.py:84-94: w = mean phi(data_pi) - phi_e; returns w.w."""
        _, tot = self.map.embed(data_pi)
        return self.fit_w(tot, data_pi.shape[0])

    def _values(self, phi: torch.Tensor, disc: torch.Tensor, thr: float):
        c = self.ctx
        n = phi.shape[0]
        reward = torch.empty(n, dtype=torch.float32, device=c.device)
        ipm = torch.empty(n, dtype=torch.float32, device=c.device)
        wb = torch.empty(n, dtype=torch.float32, device=c.device)
        self.reward_launch(phi.data_ptr(), phi.stride(0), disc.data_ptr(), float(thr), reward.data_ptr(),
                           ipm.data_ptr(), wb.data_ptr(), n)
        return reward, ipm, wb

    def reward_launch(self, phi, ldphi: int, disc, thr: float, reward, ipm, wb, n: int) -> None:
        """amx_mmd_reward (cost_range given) or amx_mmd_reward_raw (cost_range None) on raw
        device pointers."""
        c = self.ctx
        if self.cost_range is not None:
            N.check(c.lib.amx_mmd_reward(c.h, phi, ldphi, self.w.data_ptr(), self.feature_dim, disc, thr,
                                         self.lambda_b, self.c_min, self.c_max, reward, ipm, wb, n, c.stream),
                    "amx_mmd_reward")
        else:
            N.check(c.lib.amx_mmd_reward_raw(c.h, phi, ldphi, self.w.data_ptr(), self.feature_dim, disc,
                                             self.lambda_b, reward, ipm, wb, n, c.stream), "amx_mmd_reward_raw")

    def get_costs(self, x: torch.Tensor) -> torch.Tensor:
        """linear_cost.py:96-103: clamp(phi(x).w, c_min, c_max) [n, 1] (unclamped when
        cost_range is None)."""
        phi = self.get_rep(x)
        n = phi.shape[0]
        zeros = torch.zeros(n, dtype=torch.float32, device=self.ctx.device)
        # with lambda = 0 the kernel's ipm output is exactly the clamped cost
        lam, self.lambda_b = self.lambda_b, 0.0
        try:
            _, ipm, _ = self._values(phi, zeros, 1.0)
        finally:
            self.lambda_b = lam
        return ipm.view(-1, 1)

    def get_expert_cost(self) -> torch.Tensor:
        """linear_cost.py:105-109 over the resident expert features."""
        if self.cost_range is None:   # the reference clamps with c_min/c_max, unset without a range
            raise AttributeError("'RBFLinearCost' object has no attribute 'c_min'")
        c = self.ctx
        if self._expert_mean is None:
            self._expert_mean = torch.empty(1, dtype=torch.float32, device=c.device)
        if self._ear is not None:  # sharded: this rank's partial sum, all-reduced
            if not self._expert_fresh:  # w changed since the last relabel: score this rank's block
                self.wait_expert_allreduce()
                eptr, ne, _ = self._expert_args()
                N.check(c.lib.amx_expert_cost(c.h, eptr, self.expert_rep.stride(0), self.w.data_ptr(),
                                              self.feature_dim, ne, self.c_min, self.c_max,
                                              self._expert_out.data_ptr(), None, float(self.lambda_b),
                                              c.stream), "amx_expert_cost")
                self._expert_fresh, self._estate = True, "partial"
            self.expert_allreduce()   # (no-op unless the sum is still this rank's partial)
            self.wait_expert_allreduce()
            # (1 - lambda) * float32(sum / n) as k_sum_small's mean_out (the fp32 product of torch)
            torch.mul((self._expert_out[:1] / self.n_expert).float(), self._escale, out=self._expert_mean)
            return self._expert_mean[0]
        if self._expert_fresh:  # computed for the current w by the relabel launch
            return self._expert_mean[0]
        N.check(c.lib.amx_expert_cost(c.h, self.expert_rep.data_ptr(), self.expert_rep.stride(0), self.w.data_ptr(),
                                      self.feature_dim, self.n_expert, self.c_min, self.c_max,
                                      self._expert_out.data_ptr(), self._expert_mean.data_ptr(),
                                      float(self.lambda_b), c.stream), "amx_expert_cost")
        # (1 - lambda) * mean in fp32 as the reference's torch expression; a 0-dim view of a
        # persistent buffer, overwritten by the next call
        return self._expert_mean[0]

    def get_bonus_costs(self, states, actions, ensemble, next_states=None):
        """linear_cost.py:111-152: cost [T, 1] and the info dict."""
        x = cost_input(self.input_type, states, actions, next_states, self.motion)
        phi = self.get_rep(x)
        disc = device_discrepancy(ensemble, states, actions)
        reward, ipm, wb = self._values(phi, disc, ensemble.threshold)
        cost = -reward
        rff_cost = self.get_costs(x)
        return cost.view(-1, 1), {"bonus": wb.view(-1, 1), "ipm": ipm.view(-1, 1), "v_targ": rff_cost,
                                  "cost": cost.view(-1, 1)}


class GAILCost:
    """AMP/GAIL least-squares discriminator cost, inference surface (gail_cost.py:44-279)."""

    def __init__(self, expert_data: torch.Tensor, agent_rb=None, feature_dim: int = 1, hidden_dims=(1024, 512),
                 input_type: str = "ss", scaling_coef: float = 0.5, reg_coef: float = 0.05, lambda_b: float = 0.5,
                 seed=100, grad_lambda=10.0, disc_loss_type="least_squares", disc_opt="sgd", disc_opt_args=None,
                 ctx: AmxContext | None = None, device="cuda", gemm: str = "f16x3", motion=None):
        """`motion` (a ReferenceMotion) is needed for input_type "amp" (discriminator on AMP
        observations); any disc_loss_type other than "least_squares" selects the
        log-likelihood cost, as in the reference's get_costs (gail_cost.py:246-251).  `gemm`:
        the discriminator layers' GEMM ("f16x3", "bf16x6" or "f32", as DeviceEnsemble)."""
        _check_input_type(input_type, motion)
        if feature_dim != 1:
            raise ValueError("Discriminator output must be 1-D")
        torch.manual_seed(seed)          # gail_cost.py:62-63
        np.random.seed(seed)
        self.expert_data = expert_data
        self.input_dim = expert_data.size(1)
        self.input_type = input_type
        self.motion = motion
        self.lambda_b = float(lambda_b)
        self.disc_loss_type = disc_loss_type
        self.loss_code = N.AMX_DISC_LEAST_SQUARES if disc_loss_type == "least_squares" else N.AMX_DISC_LOG_LIKELIHOOD
        sizes = [self.input_dim] + list(hidden_dims) + [1]
        layers = [nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)]   # Discriminator :28-37
        for lin in layers:                                                             # disc_weight_init :11-16
            if lin.out_features == 1:
                nn.init.uniform_(lin.weight.data, a=-1.0, b=1.0)
            else:
                nn.init.xavier_uniform_(lin.weight.data)
        self.weights = [(l.weight.data.clone(), l.bias.data.clone()) for l in layers]
        if ctx is None:
            S = self.input_dim // 2 if input_type == "ss" else self.input_dim
            ctx = AmxContext(S, 1, n_models=1, hidden=128, n_hidden=0, feat_dim=128, device=device)
        self.ctx = ctx
        if gemm not in ("f16x3", "bf16x6", "f32"):
            raise ValueError(f"gemm must be 'f16x3', 'bf16x6' or 'f32', got {gemm!r}")
        self.gemm = gemm
        self.load_weights(self.weights)

    def load_weights(self, weights) -> None:
        """Upload discriminator weights (e.g. after an out-of-scope training step)."""
        dev = self.ctx.device
        self.Kin = round_up(self.input_dim, 32)
        self.dev_layers = []
        k_in, k_pad = self.input_dim, self.Kin
        for (W, b) in weights[:-1]:
            out = W.shape[0]
            out_p = round_up(out, 128)
            Wp = torch.zeros(out_p, k_pad, dtype=torch.float32)
            Wp[:out, :k_in] = W.float().cpu()
            bp = torch.zeros(out_p, dtype=torch.float32)
            bp[:out] = b.float().cpu()
            Wd = Wp.to(dev).contiguous()
            W3 = None
            if self.gemm == "bf16x6":
                W3 = split_bf16x3(self.ctx, Wd.unsqueeze(0))[0]
            elif self.gemm == "f16x3":
                W2, wexp = split_f16x2(self.ctx, Wd.unsqueeze(0))
                W3 = (W2[0], wexp[0])
            self.dev_layers.append((Wd, bp.to(dev).contiguous(), out_p, k_pad, W3))
            k_in, k_pad = out, out_p
        W3, b3 = weights[-1]
        w3 = torch.zeros(k_pad, dtype=torch.float32)
        w3[:k_in] = W3.float().cpu().view(-1)
        self.w3 = w3.to(dev).contiguous()
        self.b3 = float(b3.float().cpu().view(-1)[0])
        self.h_last = k_pad
        self._ws = {}

    def _hidden(self, x_pad: torch.Tensor, rows: int, row_exp: torch.Tensor | None = None) -> torch.Tensor:
        """Hidden layers over `rows` padded input rows.  f16x3: `row_exp` [rows] int32 = the
        input rows' exponents (amx_step_rexp for the rollout's [s, s'] rows; None computes them);
        each layer's epilogue writes the exponents of its output rows for the next."""
        c = self.ctx
        ws = self._ws.get(rows)
        if ws is None:
            ws = [torch.empty(rows, L[2], dtype=torch.float32, device=c.device) for L in self.dev_layers]
            ws.append(torch.empty(len(self.dev_layers) + 1, rows, dtype=torch.int32, device=c.device))
            self._ws[rows] = ws
        h = x_pad
        if self.gemm == "f16x3":
            rexp = ws[-1]
            if row_exp is None:
                N.check(c.lib.amx_row_exponents(c.h, 1, rows, self.Kin, h.data_ptr(), h.stride(0), 0, rexp.data_ptr(),
                                                rows, 1, c.stream), "amx_row_exponents(disc)")
                src = rexp[0]
            else:
                src = row_exp
            rexp[1:].fill_(-100)
            for i, ((Wp, bp, out_p, k_pad, (W2, wexp)), o) in enumerate(zip(self.dev_layers, ws)):
                N.check(c.lib.amx_gemm_bias_act_h3(c.h, 1, rows, out_p, k_pad, h.data_ptr(), h.stride(0), 0,
                                                   W2.data_ptr(), 0, wexp.data_ptr(), 0, bp.data_ptr(), 0,
                                                   o.data_ptr(), out_p, 0, 0, N.AMX_ACT_RELU, src.data_ptr(), 0, 1,
                                                   rexp[i + 1].data_ptr(), 0, c.stream),
                        "amx_gemm_bias_act_h3(disc)")
                h, src = o, rexp[i + 1]
            return h
        for (Wp, bp, out_p, k_pad, W3), o in zip(self.dev_layers, ws):
            if W3 is not None:
                N.check(c.lib.amx_gemm_bias_act_x6(c.h, 1, rows, out_p, k_pad, h.data_ptr(), h.stride(0), 0,
                                                   W3.data_ptr(), 0, bp.data_ptr(), 0, o.data_ptr(), out_p, 0, 0,
                                                   N.AMX_ACT_RELU, c.stream), "amx_gemm_bias_act_x6(disc)")
            else:
                N.check(c.lib.amx_gemm_bias_act(c.h, 1, rows, out_p, k_pad, h.data_ptr(), h.stride(0), 0,
                                                Wp.data_ptr(), k_pad, 0, bp.data_ptr(), 0, o.data_ptr(), out_p, 0, 0,
                                                N.AMX_ACT_RELU, c.stream), "amx_gemm_bias_act(disc)")
            h = o
        return h

    def rewards_from_input(self, x_pad: torch.Tensor, rows: int, n: int, disc: torch.Tensor | None,
                           out: torch.Tensor | None = None, logits: torch.Tensor | None = None,
                           loss_code: int | None = None, row_exp: torch.Tensor | None = None) -> torch.Tensor:
        """Fused discriminator + reward on already padded input rows [rows, Kin]."""
        c = self.ctx
        h = self._hidden(x_pad, rows, row_exp)
        out = torch.empty(n, dtype=torch.float32, device=c.device) if out is None else out
        N.check(c.lib.amx_disc_reward(c.h, self.loss_code if loss_code is None else loss_code, h.data_ptr(),
                                      h.stride(0), self.h_last, self.w3.data_ptr(), self.b3,
                                      None if disc is None else disc.data_ptr(), self.lambda_b, out.data_ptr(),
                                      None if logits is None else logits.data_ptr(), n, c.stream), "amx_disc_reward")
        return out

    def _pad(self, x: torch.Tensor):
        n = x.shape[0]
        rows = round_up(max(n, 1), 128)
        xp = torch.zeros(rows, self.Kin, dtype=torch.float32, device=self.ctx.device)
        xp[:n, :self.input_dim] = x.to(self.ctx.device, torch.float32)
        return xp, rows, n

    def disc_logits(self, ss: torch.Tensor) -> torch.Tensor:
        xp, rows, n = self._pad(ss)
        logits = torch.empty(n, dtype=torch.float32, device=self.ctx.device)
        self.rewards_from_input(xp, rows, n, None, logits=logits)
        return logits.view(-1, 1)

    def get_ls_costs(self, ss: torch.Tensor) -> torch.Tensor:
        """gail_cost.py:231-236: -max(0, 1 - 0.25 (1 - D)^2)  [n, 1]."""
        xp, rows, n = self._pad(ss)
        return (-self.rewards_from_input(xp, rows, n, None, loss_code=N.AMX_DISC_LEAST_SQUARES)).view(-1, 1)

    def get_ll_costs(self, ss: torch.Tensor) -> torch.Tensor:
        """gail_cost.py:238-244: logsigmoid(D)  [n, 1]."""
        xp, rows, n = self._pad(ss)
        return (-self.rewards_from_input(xp, rows, n, None, loss_code=N.AMX_DISC_LOG_LIKELIHOOD)).view(-1, 1)

    def get_costs(self, ss: torch.Tensor) -> torch.Tensor:
        """gail_cost.py:246-251."""
        return self.get_ls_costs(ss) if self.loss_code == N.AMX_DISC_LEAST_SQUARES else self.get_ll_costs(ss)

    def get_bonus_costs(self, states, actions, ensemble, next_states=None):
        """gail_cost.py:254-279: cost = (1-lambda) * input cost - lambda * disagreement."""
        x = cost_input(self.input_type, states, actions, next_states, self.motion)
        xp, rows, n = self._pad(x)
        disc = device_discrepancy(ensemble, states, actions)
        reward = self.rewards_from_input(xp, rows, n, disc)
        input_cost = self.get_costs(x)
        lam = np.float32(self.lambda_b)
        ipm = np.float32(1 - self.lambda_b) * input_cost
        bonus = lam * disc.view(-1, 1)
        cost = (-reward).view(-1, 1)
        return cost, {"bonus": bonus, "ipm": ipm, "v_targ": input_cost, "cost": cost}
