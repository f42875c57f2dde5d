"""Batched learned-dynamics rollout engine: B SimEnv lanes stepped in lock-step on one GPU.

One synchronous step (all lanes) is, in launch order on one HIP stream:
  1. policy      amx_policy_act        a_t = mean(s_t) + exp(log_std) * n      (gaussian_mlp.py:95-104)
  2. assemble    amx_assemble_input    x0 = [(s-mu)/sd, (a-mu)/sd]               (dynamics.py:225-230)
  3. ensemble    L x amx_gemm_bias_act + amx_gemm_out_unnorm (all M members)     (dynamics.py:422-433)
  4. step        amx_step              s' = s + Δ_k (fp64), done, disagreement, [s, s'] f32 (sim_env.py:140-268)
                 (amx_cost_rows for the 'sa' / 'sas' / 's' cost inputs, amx_state_amp_rows for AMP)
  5. auto-reset  amx_reset_lanes       done lanes <- reset-table row, model k+1  (sim_env.py:270-285)
The step kernel records the float32 [s, s'] cost-input row of every transition; the
reward pass runs once over all recorded transitions (`score`, at the end of `rollout` or
on demand), as one batched launch instead of one per step:
     amx_rff_features      phi(s, s') + fp64 column sums                 (linear_cost.py:64-94)
  or disc GEMMs + amx_amp_reward (AMP/GAIL path, fused reward)            (gail_cost.py:231-279)
(the reference scores transitions only in the relabel, batch_reinforce.py:103-169).  The
relabel then does the ordered fp64 sum of the feature partials -> (all-reduce across
ranks) -> w -> amx_mmd_reward over all K*B transitions -> expert cost.

Lane semantics: every lane is a persistent SimEnv; a trajectory that ends (fall/horizon)
auto-resets in the same step, exactly as `o = env.reset()` after `done` in get_samples
(sampler.py:48-65), and continues in the next rollout.  The model index follows SimEnv's
reset counter: model k = (#resets of the lane) mod M, so a lane's first trajectory uses
member 1 (sim_env.py:118, 282-283).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from . import _native as N
from .costs import GAILCost, RBFLinearCost, input_width
from .engine import DeviceEnsemble, round_up
from .humanoid import TerminationConfig
from .policy import DevicePolicy


# graph captures are "thread_local": in "global" mode a CUDA call made by ANY other thread during
# the capture (an RCCL process group's watchdog polling its work events) can invalidate it; the
# captured rollout itself only launches onto this thread's capture stream
_CAPTURE_MODE = "thread_local"

class RolloutEngine:
    def __init__(self, ensemble: DeviceEnsemble, reset_table, lanes: int, term: TerminationConfig | None = None,
                 policy: DevicePolicy | None = None, cost=None, seed: int = 0, max_steps: int = 16,
                 eval_mode: bool = False, auto_reset: bool = True, record_means: bool = False):
        self.ens = ensemble
        self.ctx = c = ensemble.ctx
        self.term = term or TerminationConfig()
        c.set_termination(self.term)
        self.B = int(lanes)
        self.Bp = round_up(self.B, 128)
        self.K = int(max_steps)
        self.policy = policy
        self.cost = cost
        self.eval_mode = eval_mode
        self.auto_reset = auto_reset
        self.fuse_reset = True  # table resets run inside the step kernel (amx_step_reset)
        # f16x3: the policy launch writes the ensemble's x0 + row exponents (bit-identical, tested;
        # off: with the MFMA policy and a 16-threads-per-row tail the fused launch takes 28-31 us
        # against 21 + 7 us for policy + separate assembly, no gain; bench --fuse-assembly on)
        self.fuse_assembly = False
        # rollout(): step t's kernel also runs the policy (+ x0 assembly) of step t + 1 on the
        # observations it produces (amx_step_reset_act: bit-identical to the separate launches,
        # tested); needs the fused table reset and the f16x3 shared x0 slice.  Off: measured no
        # faster than the separate launches (47-56 vs 48 us per step at 8192 lanes)
        self.fuse_step_act = False
        self._act_ready = -1      # step whose action + x0 the previous step kernel already wrote
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        dev = c.device
        from .motion import ReferenceMotion
        self.motion = reset_table if isinstance(reset_table, ReferenceMotion) else None
        # motion resets draw t ~ U(0, reset_time_max) (sim_env.py:276); 0 = the clip length (:77),
        # reset_args['time_max'] with custom_time
        self.reset_time_max = 0.0
        self.table = None
        if self.motion is None:
            table = torch.as_tensor(reset_table, dtype=torch.float64)
            if table.dim() != 2 or table.shape[1] != c.S:
                raise ValueError(f"reset table must be [R, {c.S}] float64 (or a ReferenceMotion)")
            self.table = table.to(dev).contiguous()
        S, A, B, Bp, K = c.S, c.A, self.B, self.Bp, self.K
        z = lambda *shape, dt=torch.float32: torch.zeros(*shape, dtype=dt, device=dev)
        # trajectory buffers of one rollout (obs[K] carries the lane state into the next rollout)
        self.obs = z(K + 1, B, S, dt=torch.float64)
        # gym semantics (auto_reset off: the caller resets): the next observation IS the next
        # step's input, so next_obs[t] is obs[t + 1] itself (no per-step copy)
        self.next_obs = z(K, B, S, dt=torch.float64) if auto_reset else self.obs[1:]
        self.acts = z(K, B, A, dt=torch.float64)
        self.done = z(K, B, dt=torch.uint8)
        self.disc = z(K, Bp)
        self.rewards = z(K, Bp)
        self.ipm = z(K, Bp)
        self.wbonus = z(K, Bp)
        self.nonfinite = z(K, B, dt=torch.uint8)
        self.num_steps = z(B, dt=torch.int32)
        self.steps0 = z(B, dt=torch.int32)  # in-trajectory position of slot 0 (value features)
        self.model_idx = z(B, dt=torch.int32)
        self.reset_count = z(B, dt=torch.int32)
        self.reset_rows = z(K, B, dt=torch.int32)
        self.reset_times = z(K, B, dt=torch.float64) if self.motion is not None else None
        # cost-input rows of every recorded transition, scored in one batched pass: [s, s']
        # ('ss', written by the step kernel) or [s, a], [s, a, s'], [s], AMP(s, s')
        # (amx_cost_rows after the step)
        self.cost_type = getattr(cost, "input_type", "ss") if cost is not None else "ss"
        if isinstance(cost, RBFLinearCost):
            self.kc = cost.map.Kp
        elif isinstance(cost, GAILCost):
            self.kc = cost.Kin
        else:
            self.kc = c.k_rff_pad
        if cost is not None:
            width = input_width(self.cost_type, S, A, getattr(cost, "motion", None))
            if cost.input_dim != width:
                raise ValueError(f"cost input width {cost.input_dim} does not match input_type "
                                 f"{self.cost_type!r} (S={S}, A={A}: {width})")
        self.cost_in = z(K, Bp, self.kc)
        if self.cost_type == "amp" and cost.motion.ctx is not c:
            raise ValueError("the cost's ReferenceMotion must live on the engine's context")
        # rows t*Bp + b with b >= B are padding: excluded from the feature sums
        self.row_mask = None
        if B != Bp:
            self.row_mask = ((torch.arange(K * Bp, device=dev) % Bp) < B).to(torch.uint8)
        self._scored = 0  # steps of the current rollout already scored
        self.means = z(K, B, A) if record_means else None
        # f16x3 RFF / discriminator GEMM: row exponents of the cost rows (the step kernel writes
        # them for 'ss'; the other input types get them in the scoring pass)
        self.cost_rexp = None
        if (isinstance(cost, RBFLinearCost) and cost.map.W2 is not None) or \
                (isinstance(cost, GAILCost) and cost.gemm == "f16x3"):
            self.cost_rexp = z(K, Bp, dt=torch.int32)
        if isinstance(cost, RBFLinearCost):
            self.phi = z(K, Bp, cost.feature_dim)
            self.partials = z(K, Bp // N.RFF_PART_ROWS, cost.feature_dim, dt=torch.float64)
        self.t = 0              # steps taken in the current rollout
        self.step_counter = 0   # global step counter (policy RNG stream)
        # graph mode: the counter of a captured rollout's step t is dev_step[0] + t, and the graph
        # advances dev_step by T at its end, so every replay draws fresh noise
        self.dev_step = torch.zeros(1, dtype=torch.int64, device=dev)
        self._capturing = False
        self._ctr_delta = 0      # graph capture: steps of the captured rollout (counter advance)
        self._ctr_folded = False  # the last captured step kernel advanced the counter
        self._carry = 0           # rollout(): slot holding the carried lane states (0: in slot 0)
        self._pending = None      # rollout_overlapped: the previous rollout's relabel, run at the next step 0
        self._graph_ahead = False  # replays advanced dev_step past the host counter
        # [sum phi (F) | count] of the rollout: the one buffer the cross-rank all-reduce touches
        self._fbuf = z(cost.feature_dim + 1, dt=torch.float64) if isinstance(cost, RBFLinearCost) else None
        if self._fbuf is not None:  # feature_sum()'s output is the message's first F slots
            self.phi_sum = self._fbuf[:cost.feature_dim]  # (the global sums once all-reduced)
        self.mb_mmd = None
        # rollout(): score each step's cost rows on a side stream under the next step's policy
        # (bit-identical; see rollout)
        self.score_overlap = False
        self._side = None
        # member-blocked stepping (the reference-semantics sampler): Bq > 0 = the lanes are M
        # blocks of Bq and lane b steps through member b // Bq only (DeviceEnsemble.forward_blocked;
        # its trajectory was reset onto that member), without the per-step disagreement
        self.member_blocks = 0

    # ------------------------------------------------------------------------------------
    def reset_all(self, rows: torch.Tensor | None = None) -> None:
        """SimEnv.reset on every lane (sim_env.py:270-285)."""
        self.reset_lanes(None, rows)

    def set_reset_noise(self, reset_args: dict | None) -> None:
        """SimEnv reset_args' AddNoise options for this engine's motion resets (run.py:113-117):
        None or no noise -> the plain reset.  Needs a ReferenceMotion reset source (the noise
        perturbs the kinematic pose and velocity; a reset-state table has neither)."""
        noise = N.ResetNoise.from_reset_args(reset_args) if reset_args is not None else None
        if noise is not None and self.motion is None:
            raise NotImplementedError("reset noise needs a ReferenceMotion reset source (AddNoise perturbs the "
                                      "kinematic pose / velocity, which a reset-state table does not hold)")
        self._reset_noise = noise

    def _reset_motion(self, mask, times, src, dst, t_out) -> None:
        c = self.ctx
        noise = getattr(self, "_reset_noise", None)
        N.check(c.lib.amx_reset_lanes_motion_noise(c.h, None if mask is None else mask.data_ptr(),
                                                   None if times is None else times.data_ptr(), self.seed,
                                                   float(self.reset_time_max), self.motion.kernel_flags,
                                                   None if noise is None else C.byref(noise), None, 0,
                                                   src.data_ptr(), dst.data_ptr(),
                                                   self.num_steps.data_ptr(), self.model_idx.data_ptr(),
                                                   self.reset_count.data_ptr(),
                                                   None if t_out is None else t_out.data_ptr(),
                                                   self.B, c.stream), "amx_reset_lanes_motion_noise")

    def reset_lanes(self, mask: torch.Tensor | None, rows: torch.Tensor | None = None) -> None:
        """SimEnv.reset on the lanes with mask != 0 (all lanes when mask is None); the lane
        states are taken from (and written back to) slot 0 of a fresh rollout.  With a
        ReferenceMotion reset source, `rows` are motion times [B] float64 (None: drawn
        uniform(0, duration) per lane from Philox)."""
        c = self.ctx
        self.begin_rollout()
        dst = self.obs[0]
        if self.motion is not None:
            self._reset_motion(mask, rows, dst, dst, None)
            self.t = 0
            return
        N.check(c.lib.amx_reset_lanes(c.h, None if mask is None else mask.data_ptr(), self.table.data_ptr(),
                                      self.table.shape[0], None if rows is None else rows.data_ptr(), self.seed,
                                      dst.data_ptr(), dst.data_ptr(), self.num_steps.data_ptr(),
                                      self.model_idx.data_ptr(), self.reset_count.data_ptr(), None, self.B,
                                      c.stream), "amx_reset_lanes")
        self.t = 0

    def _rollout_begin(self) -> None:
        """rollout()'s start: with the fused step the first step reads the carried lane states
        where the last rollout left them (ob_rec records them in slot 0), else begin_rollout."""
        fused = self.auto_reset and self.motion is None and self.fuse_reset
        if fused and self.t != 0:
            self._carry, self.t, self._scored = self.t, 0, 0
        else:
            self.begin_rollout()

    def begin_rollout(self) -> None:
        """Carry the lane states of the previous rollout into slot 0."""
        if self.t != 0:
            self.obs[0].copy_(self.obs[self.t])
        self.t = 0
        self._scored = 0

    def step(self, actions: torch.Tensor | None = None, reset_rows: torch.Tensor | None = None,
             noise: torch.Tensor | None = None, act_next: bool = False) -> int:
        """One synchronous step of all lanes; returns the slot index t it was recorded in.
        `actions` [B, A] f64 on device replaces the policy; `noise` [B, A] f64 replaces the
        policy's Philox noise; `reset_rows` [B] i32 forces the rows of lanes that reset.
        `act_next` (rollout()): the step kernel also computes step t + 1's policy action and
        ensemble input (amx_step_reset_act) when the configuration allows it.
        A relabel left pending by rollout_overlapped runs between the first step's ensemble
        forward and its step kernel (the forward hides the all-reduce it waits for)."""
        front = self._step_front(actions, noise)
        if front[0] == 0 and self._pending is not None:
            pending, self._pending = self._pending, None
            pending()
        fuse = act_next and actions is None and noise is None and reset_rows is None and self._can_act_next()
        return self._step_back(front, reset_rows, act_next=fuse)

    def _can_act_next(self) -> bool:
        """amx_step_reset_act applies: policy-driven steps, the fused table reset, the f16x3 GEMM's
        shared x0 slice (the kernel writes x0 once, into model 0's rows), S <= 256."""
        return (self.fuse_step_act and self.policy is not None and self.auto_reset and self.motion is None
                and self.fuse_reset and self.ens.W2 is not None and self.ens.shared_x0
                and self.ctx.S <= 256
                and self.t + 1 < self.K)

    def _step_front(self, actions, noise):
        """Policy + ensemble forward of step t (everything before the step kernel)."""
        c, t, B = self.ctx, self.t, self.B
        if t >= self.K:
            raise RuntimeError(f"rollout buffer full ({self.K} steps): call begin_rollout()")
        s = c.stream
        fused = self.auto_reset and self.motion is None and self.fuse_reset
        if t == 0 and not fused:  # (the fused step kernel records it itself: steps0_out)
            self.steps0.copy_(self.num_steps)
        # rollout(): step 0 reads the carried lane states where the last rollout left them and
        # the step kernel records them in slot 0 (ob_rec), instead of a separate carry copy
        src = self._carry if (t == 0 and self._carry) else t
        self._carry = 0
        ob, ob_next, act = self.obs[src], self.next_obs[t], self.acts[t]
        x0_ready = False
        if self._act_ready == t and actions is None and noise is None:
            # the previous step kernel already wrote this step's action, means and x0
            x0_ready = True
            self._act_ready = -1
        elif actions is not None:
            self._act_ready = -1
            act.copy_(actions)
        else:
            self._act_ready = -1
            if self.policy is None:
                raise RuntimeError("no policy and no actions given")
            if self._graph_ahead and not self._capturing:  # continue after graph replays
                self.step_counter = int(self.dev_step.item())
                self._graph_ahead = False
            # f16x3 with the shared x0 slice: the policy launch also writes x0 (once, model 0's
            # rows) and its row exponents, as amx_assemble_input_rexp (one launch fewer per step)
            fuse_x0 = self.fuse_assembly and self.ens.W2 is not None and self.ens.shared_x0
            if not fuse_x0:
                ws = None
            elif self.member_blocks:  # (x0 + exponents in the member-blocked layout)
                ws = self.ens.workspace_blocked(self.member_blocks)
            else:
                ws = self.ens.workspace(B)
            self.policy.act(ob, B, act, t if self._capturing else self.step_counter, noise=noise,
                            eval_mode=self.eval_mode, mean_out=None if self.means is None else self.means[t],
                            counter_dev=self.dev_step if self._capturing else None,
                            x0=None if ws is None else ws["act"], row_exp=None if ws is None else ws["rexp"],
                            shared_x0=fuse_x0)
            x0_ready = fuse_x0
        if self.member_blocks:
            if self.B != self.ctx.M * self.member_blocks:
                raise ValueError("member-blocked stepping needs M * member_blocks lanes")
            return t, src, self.ens.forward_blocked(ob, act, self.member_blocks, x0_ready=x0_ready)
        preds = self.ens.forward_preds(ob, act, B, x0_ready=x0_ready)
        return t, src, preds

    def _step_back(self, front, reset_rows, act_next: bool = False) -> int:
        """Step kernel (fp64 update, termination, disagreement, cost row, reset) of step t;
        with act_next also step t + 1's policy action, means and x0 (amx_step_reset_act)."""
        c, B, s = self.ctx, self.B, self.ctx.stream
        t, src, preds = front
        fused = self.auto_reset and self.motion is None and self.fuse_reset
        ob, ob_next = self.obs[src], self.next_obs[t]
        # member stride of preds (0: member-blocked, lane b's own member at row b) and the
        # disagreement output (not formed per step when member-blocked)
        sP = 0 if self.member_blocks else preds.shape[1] * c.S
        disc = self.disc[t].data_ptr() if c.M >= 2 and not self.member_blocks else None
        if fused and act_next:  # step t + policy(t+1) + x0(t+1) in one launch
            ss = self.cost_type == "ss"
            pol, ws = self.policy, self.ens.workspace(B)
            rx = ws["rexp"]
            N.check(c.lib.amx_step_reset_act(
                c.h, preds.data_ptr(), c.S, sP, self.model_idx.data_ptr(), ob.data_ptr(),
                ob_next.data_ptr(), self.num_steps.data_ptr(), self.done[t].data_ptr(),
                disc, self.cost_in[t].data_ptr() if ss else None, self.kc,
                self.cost_rexp[t].data_ptr() if ss and self.cost_rexp is not None else None,
                self.nonfinite[t].data_ptr(), self.table.data_ptr(), self.table.shape[0], None, self.seed,
                self.obs[t + 1].data_ptr(), self.reset_count.data_ptr(), self.reset_rows[t].data_ptr(),
                self.steps0.data_ptr() if t == 0 else None, self.obs[0].data_ptr() if src != t else None,
                pol.blob.data_ptr(), pol.H1, pol.H2, pol.noise_scale.data_ptr(), pol.seed,
                (t + 1) if self._capturing else (self.step_counter + 1) & 0xFFFFFFFFFFFFFFFF,
                self.dev_step.data_ptr() if self._capturing else None, int(self.eval_mode), self.acts[t + 1].data_ptr(),
                None if self.means is None else self.means[t + 1].data_ptr(), ws["act"].data_ptr(), 0, c.ldk,
                rx.data_ptr(), rx.stride(0), rx.stride(1), rx.shape[1], B, s), "amx_step_reset_act")
            self._ctr_folded = False
            self._act_ready = t + 1
        elif fused:  # step + table reset in one pass (amx_step_reset)
            ss = self.cost_type == "ss"
            # a captured rollout's last step also advances the device policy counter by T
            # (amx_counter_add folded into the step kernel: one graph node fewer)
            last = self._capturing and self._ctr_delta and t == self._ctr_delta - 1
            ctr, ctr_delta = (self.dev_step, self._ctr_delta) if last else (None, 0)
            N.check(c.lib.amx_step_reset(c.h, preds.data_ptr(), c.S, sP, self.model_idx.data_ptr(),
                                         ob.data_ptr(), ob_next.data_ptr(), self.num_steps.data_ptr(),
                                         self.done[t].data_ptr(), disc,
                                         self.cost_in[t].data_ptr() if ss else None, self.kc,
                                         self.cost_rexp[t].data_ptr() if ss and self.cost_rexp is not None else None,
                                         self.nonfinite[t].data_ptr(), self.table.data_ptr(), self.table.shape[0],
                                         None if reset_rows is None else reset_rows.data_ptr(), self.seed,
                                         self.obs[t + 1].data_ptr(), self.reset_count.data_ptr(),
                                         self.reset_rows[t].data_ptr(), self.steps0.data_ptr() if t == 0 else None,
                                         ctr.data_ptr() if ctr is not None else None, ctr_delta,
                                         self.obs[0].data_ptr() if src != t else None, B, s),
                    "amx_step_reset")
            self._ctr_folded = ctr is not None
        elif self.cost_type == "ss" and self.cost_rexp is not None:
            N.check(c.lib.amx_step_rexp(c.h, preds.data_ptr(), c.S, sP, self.model_idx.data_ptr(),
                                        ob.data_ptr(), ob_next.data_ptr(), self.num_steps.data_ptr(),
                                        self.done[t].data_ptr(), disc,
                                        self.cost_in[t].data_ptr(), self.kc, self.cost_rexp[t].data_ptr(),
                                        self.nonfinite[t].data_ptr(), B, s), "amx_step_rexp")
        else:
            N.check(c.lib.amx_step(c.h, preds.data_ptr(), c.S, sP, self.model_idx.data_ptr(),
                                   ob.data_ptr(), ob_next.data_ptr(), self.num_steps.data_ptr(),
                                   self.done[t].data_ptr(), disc,
                                   self.cost_in[t].data_ptr() if self.cost_type == "ss" else None, self.kc,
                                   self.nonfinite[t].data_ptr(), B, s), "amx_step")
        if self.cost is not None and self.cost_type != "ss":
            self._record_cost_input(t)
        if fused:
            pass
        elif self.auto_reset and self.motion is not None:
            self._reset_motion(self.done[t], reset_rows, ob_next, self.obs[t + 1], self.reset_times[t])
        elif self.auto_reset:
            N.check(c.lib.amx_reset_lanes(c.h, self.done[t].data_ptr(), self.table.data_ptr(), self.table.shape[0],
                                          None if reset_rows is None else reset_rows.data_ptr(), self.seed,
                                          ob_next.data_ptr(), self.obs[t + 1].data_ptr(), self.num_steps.data_ptr(),
                                          self.model_idx.data_ptr(), self.reset_count.data_ptr(),
                                          self.reset_rows[t].data_ptr(), B, s), "amx_reset_lanes")
        elif ob_next.data_ptr() != self.obs[t + 1].data_ptr():  # gym semantics: the caller resets
            self.obs[t + 1].copy_(ob_next)
        self.t += 1
        self.step_counter += 1
        return t

    def _record_cost_input(self, t: int) -> None:
        """Cost-input rows of step t for the non-'ss' input types (linear_cost.py:115-127)."""
        c, B, S, A = self.ctx, self.B, self.ctx.S, self.ctx.A
        ob, nx, act = self.obs[t], self.next_obs[t], self.acts[t]
        typ = self.cost_type
        if typ == "amp":   # fp32 AMP rows straight from the two recorded states
            N.check(c.lib.amx_state_amp_rows(c.h, ob.data_ptr(), nx.data_ptr(), S, B, 0,
                                             self.cost_in[t].data_ptr(), self.kc, c.stream), "amx_state_amp_rows")
            return
        if typ == "sa":
            segs = ((ob, S, S), (act, A, A), (None, 0, 0))
        elif typ == "sas":
            segs = ((ob, S, S), (act, A, A), (nx, S, S))
        else:  # "s"
            segs = ((ob, S, S), (None, 0, 0), (None, 0, 0))
        args = []
        for x, ld, w in segs:
            args += [None if x is None else x.data_ptr(), ld, w]
        N.check(c.lib.amx_cost_rows(c.h, *args, B, self.cost_in[t].data_ptr(), self.kc, c.stream), "amx_cost_rows")

    def rollout(self, K: int | None = None) -> int:
        """K synchronous steps (default: the buffer depth), then the reward pass.  With
        `score_overlap` (K > 1, MMD cost) each step's cost rows are scored on a side stream right after
        its step kernel, under the next step's latency-bound policy and assembly launches;
        otherwise in one batched launch at the end.  Same rows, same per-row work and the same
        32-row fp64 partials: the results are bit-identical either way.  Returns K*B transitions."""
        K = self.K if K is None else K
        self._rollout_begin()
        self._act_ready = -1
        # (the MMD features only: the GAIL discriminator's GEMMs split K differently at one step's
        # row count than over the whole rollout, which changes their fp32 rounding)
        side = self._score_stream() if (self.score_overlap and K > 1 and isinstance(self.cost, RBFLinearCost)) else None
        for t in range(K):
            self.step(act_next=t + 1 < K)
            if side is not None and t + 1 < K:
                side.wait_stream(torch.cuda.current_stream(self.ctx.device))
                with torch.cuda.stream(side):
                    self.score()
        if side is not None:
            torch.cuda.current_stream(self.ctx.device).wait_stream(side)
        self.score()
        return K * self.B

    def _score_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(self.ctx.device)
        return self._side

    def score(self) -> None:
        """Features (MMD) or discriminator rewards (GAIL) of the steps recorded since the last
        call, in one launch over their T*B_pad cost-input rows."""
        c, cost, t0, t1, Bp = self.ctx, self.cost, self._scored, self.t, self.Bp
        if t1 <= t0 or cost is None:
            self._scored = t1
            return
        rows = (t1 - t0) * Bp
        x = self.cost_in[t0:t1].view(rows, self.kc)
        if isinstance(cost, RBFLinearCost):
            mask = None if self.row_mask is None else self.row_mask[t0 * Bp:t1 * Bp]
            rexp = None
            if self.cost_rexp is not None and self.cost_type == "ss":
                rexp = self.cost_rexp[t0:t1].view(rows)
            cost.map.features(x, rows, rows, self.phi[t0:t1].view(rows, -1),
                              self.partials[t0:t1].view(rows // N.RFF_PART_ROWS, -1), row_mask=mask, row_exp=rexp)
        elif isinstance(cost, GAILCost):
            rexp = None
            if self.cost_rexp is not None and self.cost_type == "ss":
                rexp = self.cost_rexp[t0:t1].view(rows)
            cost.rewards_from_input(x, rows, rows, self.disc[t0:t1].view(rows) if c.M >= 2 else None,
                                    out=self.rewards[t0:t1].view(rows), row_exp=rexp)
        self._scored = t1

    # ------------------------------------------------------------------------------------
    def feature_sum(self) -> torch.Tensor:
        """Ordered fp64 sum of this rank's RFF column partials over the recorded steps."""
        self.relabel_pre()
        return self.phi_sum

    def relabel(self, allreduce=None) -> dict:
        """Relabel the recorded transitions (batch_reinforce.py:103-169, MMD + ensemble).
        `allreduce(tensor)` sums a device tensor across ranks in place (None: one rank)."""
        cost = self.cost
        self.flush_relabel()  # a relabel rollout_overlapped left pending comes first
        self.score()
        if isinstance(cost, GAILCost):
            return {}  # rewards come from the discriminator pass
        if not isinstance(cost, RBFLinearCost):
            raise RuntimeError("relabel needs an RBFLinearCost or GAILCost")
        self.relabel_pre()
        if allreduce is not None:
            allreduce(self._fbuf)  # ONE fused all-reduce of [sum phi, count] across ranks
        return self.relabel_post()

    def relabel_pre(self) -> torch.Tensor:
        """Rank-local half of the relabel: this rank's [sum phi | count] (amx_feature_message)
        in the persistent fp64 buffer that the cross-rank all-reduce sums (dist.feature_mean's
        message); phi_sum is a view of its first F slots."""
        self.score()
        c, cost = self.ctx, self.cost
        n_parts = self.t * (self.Bp // N.RFF_PART_ROWS)
        N.check(c.lib.amx_feature_message(c.h, self.partials.data_ptr(), n_parts, cost.feature_dim,
                                          float(self.t * self.B), self._fbuf.data_ptr(), c.stream),
                "amx_feature_message")
        return self._fbuf

    def relabel_post(self, T: int | None = None) -> dict:
        """Global half, one launch (amx_mmd_relabel): mean -> witness w (the fp64 mean rounded
        to fp32, count from the message's last slot) -> per-sample rewards of every recorded
        transition (the first T steps; default: the current rollout's), and the expert cost for
        the new w."""
        cost = self.cost
        n = (self.t if T is None else T) * self.Bp
        self.mb_mmd = cost.relabel_device(self._fbuf, self.phi.data_ptr(), cost.feature_dim, self.disc.data_ptr(),
                                          float(self.ens.threshold), self.rewards.data_ptr(), self.ipm.data_ptr(),
                                          self.wbonus.data_ptr(), n)
        return {"mb_mmd": self.mb_mmd}

    def graph_rollout(self, T: int | None = None, allreduce=None, tail=None, before_relabel=None, after=None):
        """Capture one full rollout (K steps + scoring + relabel + `tail()`, e.g. the expert
        cost) as HIP graph(s) on the current device and return `replay()`; replaying it is
        equivalent to `rollout(T); relabel(allreduce); tail()` (the policy's Philox counter
        lives on the device).  With `allreduce` (several ranks) the collective stays eager
        between two graphs; `before_relabel()` runs on the host right before the relabel's graph
        and `after()` after the last one (e.g. RBFLinearCost.wait_expert_allreduce /
        expert_allreduce_replayed of a sharded expert cost).  Run one eager rollout first (workspaces
        allocated, t == T)."""
        T = self.K if T is None else T
        if self.t != T:
            raise RuntimeError("run one eager rollout(T) before capturing")
        mmd = isinstance(self.cost, RBFLinearCost)
        c = self.ctx
        if self._graph_ahead:
            self.step_counter = int(self.dev_step.item())
        self.dev_step.fill_(self.step_counter)  # the counter the next eager step would use
        graphs = [torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()]
        side = torch.cuda.Stream(c.device)
        side.wait_stream(torch.cuda.current_stream(c.device))
        with torch.cuda.stream(side):
            self._capturing = True
            self._ctr_delta, self._ctr_folded = T, False
            try:
                with torch.cuda.graph(graphs[0], stream=side, capture_error_mode=_CAPTURE_MODE):
                    self.rollout(T)
                    if not self._ctr_folded:  # (the fused step kernel advances it itself)
                        N.check(c.lib.amx_counter_add(c.h, self.dev_step.data_ptr(), T, c.stream), "amx_counter_add")
                    if mmd:
                        self.relabel_pre()
                        if allreduce is None:
                            self.relabel_post()
                    if tail is not None and (allreduce is None or not mmd):
                        tail()
                if mmd and allreduce is not None:
                    with torch.cuda.graph(graphs[1], stream=side, capture_error_mode=_CAPTURE_MODE):
                        self.relabel_post()
                        if tail is not None:
                            tail()
            finally:
                self._capturing = False
                self._ctr_delta = 0
        torch.cuda.current_stream(c.device).wait_stream(side)
        self._graph_ahead = True  # the captured steps did not run: the device counter is the truth
        two = mmd and allreduce is not None

        def replay():
            graphs[0].replay()
            if two:
                if before_relabel is not None:
                    before_relabel()
                allreduce(self._fbuf)
                graphs[1].replay()
            if after is not None:
                after()
            self._graph_ahead = True
            return T * self.B
        return replay

    def rollout_overlapped(self, T: int, allreduce_async, tail=None) -> int:
        """One rollout of T steps whose cross-rank all-reduce overlaps the NEXT rollout's first
        ensemble forward (multi-rank MMD path): the rollout's [sum phi | count] message is
        handed to `allreduce_async(buf)` (returns a handle with .wait(): e.g.
        dist.all_reduce(async_op=True), which queues the GPU-side wait), and its relabel
        (relabel_post + `tail()`) runs at the next rollout's step 0, between the forward and the
        step kernel -- nothing the forward launches reads or writes the relabel's buffers
        (phi, disc, the message, rewards).  flush_relabel() completes the last one.  The
        results equal rollout(T); relabel(allreduce); tail() per rollout.  Valid while the
        rollouts share the policy (fixed-policy collection, evaluation): a trainer that updates
        the policy from one rollout's rewards before the next uses rollout + relabel."""
        if not isinstance(self.cost, RBFLinearCost):
            raise RuntimeError("rollout_overlapped is the MMD path (RBFLinearCost)")
        self.rollout(T)
        self.relabel_pre()
        h = allreduce_async(self._fbuf)

        def pending():
            h.wait()
            self.relabel_post(T)
            if tail is not None:
                tail()
        self._pending = pending
        return T * self.B

    def flush_relabel(self) -> None:
        """Run the relabel rollout_overlapped left pending (no-op when none is)."""
        if self._pending is not None:
            pending, self._pending = self._pending, None
            pending()

    def graph_rollout_overlapped(self, T: int, allreduce_async, tail=None, before_relabel=None, after=None):
        """rollout_overlapped as HIP graphs: G0 = the first step's policy + forward, G1 = the
        previous rollout's relabel + tail, the first step kernel, steps 1..T-1, scoring and the
        message; the all-reduce is issued between replays and waited for (GPU-side) only
        before G1, so it runs under the next G0.  Returns (replay, flush): replay() runs one
        rollout, flush() waits for the last all-reduce and runs its relabel (graph G2).  Run
        one eager rollout + relabel first (t == T; its relabel is recomputed by the first
        replay's G1, unchanged).  `before_relabel()` / `after()`: host hooks around the graphs
        holding a relabel (as graph_rollout's)."""
        if not isinstance(self.cost, RBFLinearCost):
            raise RuntimeError("graph_rollout_overlapped is the MMD path (RBFLinearCost)")
        if self.t != T or self._pending is not None:
            raise RuntimeError("run one eager rollout(T) + relabel before capturing")
        fused = self.auto_reset and self.motion is None and self.fuse_reset
        if not fused:
            raise RuntimeError("graph_rollout_overlapped needs the fused step + table reset")
        c = self.ctx
        if self._graph_ahead:
            self.step_counter = int(self.dev_step.item())
        self.dev_step.fill_(self.step_counter)
        graphs = [torch.cuda.CUDAGraph() for _ in range(3)]
        side = torch.cuda.Stream(c.device)
        side.wait_stream(torch.cuda.current_stream(c.device))
        with torch.cuda.stream(side):
            self._capturing = True
            self._ctr_delta, self._ctr_folded = T, False
            try:
                with torch.cuda.graph(graphs[0], stream=side, capture_error_mode=_CAPTURE_MODE):
                    self._rollout_begin()
                    front = self._step_front(None, None)
                with torch.cuda.graph(graphs[1], stream=side, capture_error_mode=_CAPTURE_MODE):
                    self.relabel_post(T)
                    if tail is not None:
                        tail()
                    self._step_back(front, None)
                    for _ in range(T - 1):
                        self.step()
                    self.score()
                    if not self._ctr_folded:
                        N.check(c.lib.amx_counter_add(c.h, self.dev_step.data_ptr(), T, c.stream), "amx_counter_add")
                    self.relabel_pre()
                with torch.cuda.graph(graphs[2], stream=side, capture_error_mode=_CAPTURE_MODE):
                    self.relabel_post(T)
                    if tail is not None:
                        tail()
            finally:
                self._capturing = False
                self._ctr_delta = 0
        torch.cuda.current_stream(c.device).wait_stream(side)
        self._graph_ahead = True
        state = {"h": None}

        def replay():
            graphs[0].replay()
            if state["h"] is not None:
                state["h"].wait()
            if before_relabel is not None:
                before_relabel()
            graphs[1].replay()
            state["h"] = allreduce_async(self._fbuf)
            if after is not None:
                after()
            self._graph_ahead = True
            return T * self.B

        def flush():
            if state["h"] is not None:
                state["h"].wait()
                state["h"] = None
                if before_relabel is not None:
                    before_relabel()
                graphs[2].replay()
                if after is not None:
                    after()
        return replay, flush

    def advantages(self, baseline, gamma: float = 0.995, gae_lambda=0.97, whiten: bool = False,
                   eps: float = 1e-6) -> dict:
        """Returns, baseline values and GAE advantages of the recorded steps
        (process_samples.py:3-35 over the lane buffers): trajectories end at done flags
        (terminated: bootstrap 0); a lane's trajectory still running at the end of the buffer
        is bootstrapped with its last baseline value (mjrl's non-terminated rule).
        `whiten` applies process_paths' (adv - mean) / (std + eps) (batch_reinforce.py:284-285).
        All outputs are device tensors [T, B] (values f32, returns/advantages f64)."""
        from .gae import gae_grid, whiten_grid
        self.flush_relabel()  # the rewards of a relabel rollout_overlapped left pending
        c, T, B = self.ctx, self.t, self.B
        rows = T * B
        obs = self.obs[:T].reshape(rows, c.S)
        end = self.done[:T].reshape(rows)
        v = baseline.predict_grid(rows, T, B, obs, c.S, end, B, t0=self.steps0)
        ret = torch.empty(T, B, dtype=torch.float64, device=c.device)
        adv = torch.empty_like(ret)
        gae_grid(c, T, B, end, self.rewards, self.Bp, v, gamma, gae_lambda, B, ret, adv)
        out = {"values": v[:rows].view(T, B), "returns": ret, "advantages": adv}
        if whiten:
            out["advantages_whitened"], out["adv_stats"] = whiten_grid(c, T, B, adv, B, eps=eps,
                                                                       out=torch.empty_like(adv))
        return out

    def bonus_mmd(self, allreduce=None) -> float:
        """infos['bonus_mmd'] = mean(-rewards) - expert cost (batch_reinforce.py:169).
        `allreduce` (lanes sharded over ranks, as for relabel): the mean over every rank's
        samples, from one all-reduce of the fp64 [sum, count] pair (SURVEY §8(e)'s logging
        scalars); the expert cost is already global (one rank's shard sum all-reduced, or
        every rank scoring all expert rows).  With `allreduce` every rank must call it (it is a
        collective)."""
        self.flush_relabel()  # the rewards of a relabel rollout_overlapped left pending
        T, B = self.t, self.B
        cost = -self.rewards[:T, :B].double()
        if allreduce is None:
            mean_cost = cost.mean()
        else:
            m = torch.stack([cost.sum(), torch.full((), float(T * B), dtype=torch.float64, device=cost.device)])
            allreduce(m)
            mean_cost = m[0] / m[1]
        return float(mean_cost.item()) - float(self.cost.get_expert_cost().item())
