"""Device-resident building blocks over the amx C ABI: context, the dense-MLP ensemble,
RFF features and the reward kernels.

Layout in HBM (all fp32 unless noted; B_pad = round_up(B, 128)):
  act   [M][B_pad][ldk]     dense-concat activation rows: [s~, a~, 0-pad | h0 | h1 | h2 | h3]
                            (ldk = k0_pad + L*Hp; k0_pad = round_up(S+A, 32))
  W_i   [M][Hp][k0_pad+i*Hp] hidden-layer weights re-indexed into that column layout
  W_out [M][n_out_pad][ldk]  last layer, rows >= S zero
  preds [M][B_pad][S]        un-normalised state deltas of every member
Hidden widths that are not multiples of 128 are zero-padded (ReLU(0) = 0 keeps the pad
inert), so any BasicMLP config runs on the same 128x128 MFMA tiles.
"""
from __future__ import annotations


import numpy as np
import torch

from . import _native as N
from .humanoid import TerminationConfig


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class AmxContext:
    """One amx_ctx per device (include/amx_hip.h)."""

    def __init__(self, S: int, A: int, n_models: int = 4, hidden: int = 512, n_hidden: int = 4,
                 feat_dim: int = 512, device: torch.device | str | int = "cuda"):
        self.lib = N.load()
        self.device = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
        if self.device.type != "cuda":
            raise N.AmxNativeError("the amx engine runs on a ROCm GPU only (no CPU path)")
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        self.S, self.A, self.M = S, A, n_models
        self.Hp = round_up(hidden, 128)
        self.L = n_hidden
        self.F = round_up(feat_dim, 128)
        with torch.cuda.device(idx):
            h = self.lib.amx_create(idx, S, A, n_models, self.Hp, n_hidden, self.F)
        if not h:
            raise N.AmxNativeError("amx_create failed: " + self.lib.amx_last_error().decode())
        self.h = h
        # device buffers registered with the context (split-K workspaces, timers): captured HIP
        # graphs bake their pointers into kernel arguments, so none is ever freed before the context
        self._retained = []
        k0, ldk, nout, kr = (N.C.c_int(), N.C.c_int(), N.C.c_int(), N.C.c_int())
        N.check(self.lib.amx_layout(h, N.C.byref(k0), N.C.byref(ldk), N.C.byref(nout), N.C.byref(kr)), "amx_layout")
        self.k0_pad, self.ldk, self.n_out_pad, self.k_rff_pad = k0.value, ldk.value, nout.value, kr.value
        # compute units (the C side's tile choices use the same device property)
        self.n_cus = torch.cuda.get_device_properties(self.device).multi_processor_count

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.amx_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def gemm_timer(self, on: bool = True):
        """In-kernel timing of the f16x3 ensemble forwards (amx_set_gemm_timer): returns the
        device buffer [start, arrivals, ticks (100 MHz), forwards], zeroed; off with on=False."""
        if not on:
            N.check(self.lib.amx_set_gemm_timer(self.h, None), "amx_set_gemm_timer")
            return None
        self._timer = torch.zeros(4, dtype=torch.int64, device=self.device)
        # graphs captured while an earlier timer was registered keep writing to it: every
        # buffer ever handed to the context lives as long as the context
        self._retained.append(self._timer)
        N.check(self.lib.amx_set_gemm_timer(self.h, self._timer.data_ptr()), "amx_set_gemm_timer")
        return self._timer

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def set_normalizers(self, norms) -> None:
        arrs = [np.ascontiguousarray(torch.as_tensor(x).detach().cpu().float().numpy()) for x in norms]
        assert arrs[0].shape == (self.S,) and arrs[2].shape == (self.A,) and arrs[4].shape == (self.S,)
        self._norm_host = arrs  # keep alive during the (synchronous) copy
        N.check(self.lib.amx_set_normalizers(self.h, *[a.ctypes.data for a in arrs]), "amx_set_normalizers")

    def set_termination(self, cfg: TerminationConfig) -> None:
        ids, shapes, p0, p1 = cfg.tables()
        ids_a = np.ascontiguousarray(ids, dtype=np.int32)
        sh_a = np.ascontiguousarray(shapes, dtype=np.int32)
        p0_a = np.ascontiguousarray(p0, dtype=np.float64)
        p1_a = np.ascontiguousarray(p1, dtype=np.float64)
        N.check(self.lib.amx_set_termination(
            self.h, len(ids), ids_a.ctypes.data, sh_a.ctypes.data, p0_a.ctypes.data, p1_a.ctypes.data,
            int(cfg.record_all_world), int(cfg.record_world_root_pos), cfg.pos_dim, cfg.rot_dim, int(cfg.horizon),
            int(cfg.enable_velocity_check), int(cfg.vel_offset), float(cfg.vel_threshold),
            int(cfg.record_vel_as_pos), float(cfg.sampling_rate)), "amx_set_termination")

    # ---- thin checked launchers -------------------------------------------------------
    def gemm_bias_act(self, groups, rows, Nn, K, A, lda, sA, W, ldw, sW, bias, sB, C, ldc, sC, col_off, act):
        N.check(self.lib.amx_gemm_bias_act(self.h, groups, rows, Nn, K, A.data_ptr(), lda, sA, W.data_ptr(), ldw, sW,
                                           bias.data_ptr(), sB, C.data_ptr(), ldc, sC, col_off, act, self.stream),
                "amx_gemm_bias_act")


def split_bf16x3(ctx: AmxContext, W: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """3-limb bf16 image [G][rows][K/16][3][16] (int16 bits) of a [G][rows][K] fp32 device
    weight (amx_split_bf16x3), the operand of the amx_*_x6 GEMMs; `out` rewrites an image in place."""
    G, rows, K = W.shape
    W = W.contiguous()
    W3 = torch.empty(G, rows, 3 * K, dtype=torch.int16, device=ctx.device) if out is None else out
    _check_dev(W3, torch.int16, "out", ctx.device)
    if tuple(W3.shape) != (G, rows, 3 * K):
        raise ValueError(f"out: expected shape {(G, rows, 3 * K)}, got {tuple(W3.shape)}")
    N.check(ctx.lib.amx_split_bf16x3(ctx.h, G, rows, K, W.data_ptr(), K, rows * K, W3.data_ptr(), rows * 3 * K,
                                     ctx.stream), "amx_split_bf16x3")
    return W3


def split_f16x2(ctx: AmxContext, W: torch.Tensor, out=None):
    """Scaled 2-limb fp16 image [G][rows][K/16][2][16] (int16 bits) + row exponents [G][rows]
    of a [G][rows][K] fp32 device weight (amx_split_f16x2), the operand of the amx_*_h3 GEMMs;
    `out` = (image, exponents) rewrites an existing pair in place."""
    G, rows, K = W.shape
    W = W.contiguous()
    if out is None:
        W2 = torch.empty(G, rows, 2 * K, dtype=torch.int16, device=ctx.device)
        wexp = torch.empty(G, rows, dtype=torch.int32, device=ctx.device)
    else:
        W2, wexp = out
        _check_dev(W2, torch.int16, "out[0]", ctx.device)
        _check_dev(wexp, torch.int32, "out[1]", ctx.device)
        if tuple(W2.shape) != (G, rows, 2 * K) or tuple(wexp.shape) != (G, rows):
            raise ValueError(f"out: expected shapes {(G, rows, 2 * K)} and {(G, rows)}, got "
                             f"{tuple(W2.shape)} and {tuple(wexp.shape)}")
    N.check(ctx.lib.amx_split_f16x2(ctx.h, G, rows, K, W.data_ptr(), K, rows * K, W2.data_ptr(), rows * 2 * K,
                                    wexp.data_ptr(), rows, ctx.stream), "amx_split_f16x2")
    return W2, wexp


def _check_dev(t: torch.Tensor, dtype, name: str, device) -> None:
    if not isinstance(t, torch.Tensor) or t.device != device or t.dtype != dtype or not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous {dtype} tensor on {device}, got "
                         f"{getattr(t, 'dtype', type(t))} on {getattr(t, 'device', '?')}")


class DeviceEnsemble:
    """The dense-connect BasicMLP ensemble resident in HBM (milo/milo/dynamics.py:19-233).

    `weights[m]` = [(W0, b0), ..., (WL, bL)] in nn.Linear layout (W [out, in]); `norms` =
    the 6 transformation vectors of AmpDataset.get_transformations (datasets.py:23-43).
    All members share the normalizers (DynamicsEnsemble.load_ensemble, dynamics.py:128-131).
    """

    GEMM_PRECISIONS = ("f16x3", "bf16x6", "f32")

    def __init__(self, ctx: AmxContext, weights, norms, threshold: float = 0.0, gemm: str = "f16x3"):
        """gemm: "bf16x6" (fp32 operands split into 3 bf16 limbs, 6 limb products on the bf16
        MFMA pipe: fp32-level error, amx_gemm_*_x6), "f16x3" (power-of-two scaled operands
        split into 2 fp16 limbs, 3 products; the default) or "f32" (v_mfma_f32_32x32x2_f32)."""
        if gemm not in self.GEMM_PRECISIONS:
            raise ValueError(f"gemm must be one of {self.GEMM_PRECISIONS}, got {gemm!r}")
        self.gemm = gemm
        # exponent slots per row (f16x3): x0, h0 .. h_{L-1}
        self.n_slots = ctx.L + 1
        self.shared_x0 = True  # f16x3: x0 assembled once, read by every member (k_shared)
        self.ctx = ctx
        M, Hp, L = ctx.M, ctx.Hp, ctx.L
        if len(weights) != M:
            raise ValueError(f"expected {M} ensemble members, got {len(weights)}")
        hidden = weights[0][0][0].shape[0]
        self.hidden = hidden
        if round_up(hidden, 128) != Hp or len(weights[0]) != L + 1:
            raise ValueError("weights do not match the context's (hidden, n_hidden)")
        self.W = self.b = self.W3 = self.W2 = self.wexp = None
        self.set_weights(weights)
        ctx.set_normalizers(norms)
        self.norms = tuple(torch.as_tensor(x).float().to(ctx.device) for x in norms)
        self.threshold = float(threshold)
        self._ws = {}
        # optional timing hook: when a list, every forward appends a (start, end) pair of
        # torch.cuda.Events recorded on the launch stream around the L+1 GEMM launches (inside
        # captured graphs use the context's in-kernel timer instead: AmxContext.gemm_timer)
        self.gemm_events = None

    def set_weights(self, weights) -> None:
        """(Re)load the members' nn.Linear weights, re-indexed into the dense-concat column
        layout and split into the GEMM path's limb image.  After the first call the device
        buffers are updated in place, so engines and captured graphs that hold their pointers
        see the new weights (DynamicsEnsemble.load_ensemble, dynamics.py:118-131)."""
        ctx = self.ctx
        S, A, M, Hp, L = ctx.S, ctx.A, ctx.M, ctx.Hp, ctx.L
        if len(weights) != M:
            raise ValueError(f"expected {M} ensemble members, got {len(weights)}")
        hidden = self.hidden
        dev, k0 = ctx.device, ctx.k0_pad
        # original input column -> padded activation column
        colmap = np.concatenate([np.arange(S + A)] + [k0 + i * Hp + np.arange(hidden) for i in range(L)])
        Ws, bs = [], []
        for i in range(L + 1):
            last = i == L
            n_rows = ctx.n_out_pad if last else Hp
            Kp = ctx.ldk if last else k0 + i * Hp
            Wp = torch.zeros(M, n_rows, Kp, dtype=torch.float32)
            bp = torch.zeros(M, n_rows, dtype=torch.float32)
            for m in range(M):
                if len(weights[m]) != L + 1:
                    raise ValueError(f"member {m}: {len(weights[m])} layers, expected {L + 1}")
                W_m, b_m = weights[m][i]
                W_m = torch.as_tensor(W_m).detach().float().cpu()
                out_dim, in_dim = W_m.shape
                exp_in = S + A + i * hidden
                if in_dim != exp_in or out_dim != (S if last else hidden):
                    raise ValueError(f"layer {i} of member {m}: shape {tuple(W_m.shape)}, expected "
                                     f"({S if last else hidden}, {exp_in})")
                Wp[m, :out_dim][:, torch.from_numpy(colmap[:in_dim])] = W_m
                bp[m, :out_dim] = torch.as_tensor(b_m).detach().float().cpu()
            Ws.append(Wp)
            bs.append(bp)
        if self.W is None:
            self.W = [w.to(dev).contiguous() for w in Ws]
            self.b = [b.to(dev).contiguous() for b in bs]
            if self.gemm == "bf16x6":
                self.W3 = [split_bf16x3(ctx, W) for W in self.W]
            elif self.gemm == "f16x3":
                sp = [split_f16x2(ctx, W) for W in self.W]
                self.W2, self.wexp = [x[0] for x in sp], [x[1] for x in sp]
            return
        for i in range(L + 1):
            self.W[i].copy_(Ws[i])
            self.b[i].copy_(bs[i])
            if self.W3 is not None:
                split_bf16x3(ctx, self.W[i], out=self.W3[i])
            if self.W2 is not None:
                split_f16x2(ctx, self.W[i], out=(self.W2[i], self.wexp[i]))

    @property
    def num_models(self) -> int:
        return self.ctx.M

    def workspace(self, B: int):
        """Activation + prediction buffers for B lanes (cached per B_pad).  B_pad = round_up(B, 128),
        or to 256 for large odd counts (the relabel's 40 530 samples: the 256 x 256 tiles need it)."""
        Bp = round_up(max(B, 1), 128)
        if Bp >= 16384 and Bp % 256:
            Bp += 128
        ws = self._ws.get(Bp)
        if ws is None:
            c = self.ctx
            ws = dict(Bp=Bp, act=torch.zeros(c.M, Bp, c.ldk, dtype=torch.float32, device=c.device),
                      preds=torch.zeros(c.M, Bp, c.S, dtype=torch.float32, device=c.device),
                      # f16x3: row exponents [M][slots][Bp] (x0, h0..h_{L-1})
                      rexp=torch.zeros(c.M, self.n_slots, Bp, dtype=torch.int32, device=c.device))
            if self.W2 is not None:
                self._ensure_split_workspace(Bp)
            self._ws[Bp] = ws
        return ws

    def workspace_blocked(self, Bq: int):
        """Buffers of the member-blocked forward (forward_blocked): M blocks of Bq lanes, lane
        b = g * Bq + r runs member g only.  act [1][M * Bq][ldk] (one x0 per lane), preds
        [M * Bq][S] (lane b's delta at row b), row exponents [M][slots][Bq] (the member-blocked
        exponent layout of amx_assemble_input_rexp / amx_policy_act: slot stride Bq)."""
        if Bq <= 0 or Bq % 128:
            raise ValueError(f"member blocks of {Bq} lanes: must be a positive multiple of 128")
        key = ("blocked", Bq)
        ws = self._ws.get(key)
        if ws is None:
            c = self.ctx
            ws = dict(Bq=Bq, act=torch.zeros(1, c.M * Bq, c.ldk, dtype=torch.float32, device=c.device),
                      preds=torch.zeros(c.M * Bq, c.S, dtype=torch.float32, device=c.device),
                      rexp=torch.zeros(c.M, self.n_slots, Bq, dtype=torch.int32, device=c.device))
            self._ensure_split_workspace(Bq)
            self._ws[key] = ws
        return ws

    def forward_blocked(self, ob: torch.Tensor, act: torch.Tensor, Bq: int, x0_ready: bool = False) -> torch.Tensor:
        """One member per lane: lanes [g * Bq, (g + 1) * Bq) through member g alone (SimEnv.step
        runs the lane's current member only, sim_env.py:154-157, with reset_counter % M choosing
        it at reset, :282-283).  A quarter of forward_preds' rows for the reference-semantics
        sampler, whose lanes are placed in the block of their trajectory's member.  Returns
        preds [M * Bq][S] (view of the workspace).  f16x3 only.  `x0_ready`: the policy launch
        already wrote x0 and its exponents into workspace_blocked(Bq) (amx_policy_act's fused
        assembly in the member-blocked layout)."""
        if self.W2 is None:
            raise ValueError("forward_blocked needs the f16x3 GEMM")
        c = self.ctx
        B = c.M * Bq
        if ob.dtype != act.dtype or ob.dtype not in (torch.float64, torch.float32):
            raise ValueError("ob and act must both be float64 or both float32")
        _check_dev(ob, ob.dtype, "ob", c.device)
        _check_dev(act, act.dtype, "act", c.device)
        if ob.shape[-1] != c.S or act.shape[-1] != c.A or ob.shape[0] < B or act.shape[0] < B:
            raise ValueError(f"ob {tuple(ob.shape)} / act {tuple(act.shape)} do not match S={c.S}, A={c.A}, "
                             f"{c.M} blocks of {Bq} lanes")
        ws = self.workspace_blocked(Bq)
        buf, preds, rexp = ws["act"], ws["preds"], ws["rexp"]
        s = c.stream
        dt = N.AMX_IN_F64 if ob.dtype == torch.float64 else N.AMX_IN_F32
        sA, sR, L = Bq * c.ldk, self.n_slots * Bq, c.L
        if not x0_ready:  # x0 once per lane + slot 0 of its member block's exponents (slot stride Bq)
            N.check(c.lib.amx_assemble_input_rexp(c.h, ob.data_ptr(), act.data_ptr(), dt, buf.data_ptr(), 0, c.ldk, B,
                                                  rexp.data_ptr(), sR, Bq, self.n_slots, s), "amx_assemble_input_rexp")
        for i in range(L):
            K = c.k0_pad + i * c.Hp
            N.check(c.lib.amx_gemm_bias_act_h3(c.h, c.M, Bq, c.Hp, K, buf.data_ptr(), c.ldk, sA, self.W2[i].data_ptr(),
                                               c.Hp * 2 * K, self.wexp[i].data_ptr(), c.Hp, self.b[i].data_ptr(), c.Hp,
                                               buf.data_ptr(), c.ldk, sA, K, N.AMX_ACT_RELU, rexp.data_ptr(), sR,
                                               i + 1, rexp[0, i + 1].data_ptr(), 0, s), "amx_gemm_bias_act_h3")
        N.check(c.lib.amx_gemm_out_unnorm_h3(c.h, c.M, Bq, c.S, c.ldk, buf.data_ptr(), c.ldk, sA,
                                             self.W2[L].data_ptr(), c.n_out_pad * 2 * c.ldk, self.wexp[L].data_ptr(),
                                             c.n_out_pad, self.b[L].data_ptr(), c.n_out_pad, preds.data_ptr(), c.S,
                                             Bq * c.S, rexp.data_ptr(), sR, L + 1, 0, s), "amx_gemm_out_unnorm_h3")
        return preds

    def _ensure_split_workspace(self, Bp: int) -> None:
        """Register the output layer's split-K scratch with the context when Bp lanes split
        (amx_split_workspace_floats > 0); the buffer only grows.  A replaced buffer stays
        alive (AmxContext._retained): graphs captured before the growth still launch with its
        pointers, and its self-resetting arrival counters are zero between launches."""
        c = self.ctx
        nc = N.C.c_int(0)
        floats = int(c.lib.amx_split_workspace_floats(c.h, c.M, Bp, N.C.byref(nc)))
        if floats <= 0:
            return
        cur = getattr(c, "_split_ws", None)
        if cur is not None and cur[0].numel() >= floats and cur[1].numel() >= nc.value:
            return
        scratch = torch.empty(floats, dtype=torch.float32, device=c.device)
        counters = torch.zeros(max(nc.value, 1), dtype=torch.int32, device=c.device)
        N.check(c.lib.amx_set_split_workspace(c.h, scratch.data_ptr(), floats, counters.data_ptr(), nc.value),
                "amx_set_split_workspace")
        c._split_ws = (scratch, counters)
        c._retained.append(c._split_ws)

    def forward_preds(self, ob: torch.Tensor, act: torch.Tensor, B: int | None = None,
                      assembled: bool = False, x0_ready: bool = False) -> torch.Tensor:
        """All members' un-normalised deltas for rows [0, B): returns preds [M, Bp, S] (view
        of the workspace; rows >= B are padding).  ob/act fp64 or fp32 on the device.
        `x0_ready` (f16x3): the caller (amx_policy_act's fused assembly) already wrote the shared
        x0 slice into model 0's rows and the row-exponent slots of the workspace."""
        c = self.ctx
        B = ob.shape[0] if B is None else B
        if ob.dtype != act.dtype or ob.dtype not in (torch.float64, torch.float32):
            raise ValueError("ob and act must both be float64 or both float32")
        _check_dev(ob, ob.dtype, "ob", c.device)
        _check_dev(act, act.dtype, "act", c.device)
        if ob.shape[-1] != c.S or act.shape[-1] != c.A or ob.shape[0] < B or act.shape[0] < B:
            raise ValueError(f"ob {tuple(ob.shape)} / act {tuple(act.shape)} do not match S={c.S}, A={c.A}, B={B}")
        ws = self.workspace(B)
        Bp, buf, preds = ws["Bp"], ws["act"], ws["preds"]
        dt = N.AMX_IN_F64 if ob.dtype == torch.float64 else N.AMX_IN_F32
        s = c.stream
        rexp = ws["rexp"]
        k_shared = 0
        if x0_ready:
            if self.W2 is None:
                raise ValueError("x0_ready needs the f16x3 GEMM (shared x0 slice + row exponents)")
            self._mlp(buf, preds, Bp, s, rexp, row_exponents=False, k_shared=c.k0_pad)
            return preds
        if not assembled and self.W2 is not None:  # x0 + its row exponents in one pass
            # shared_x0: one x0 copy (model 0's rows) that every model's GEMMs read (k_shared)
            k_shared = c.k0_pad if self.shared_x0 else 0
            N.check(c.lib.amx_assemble_input_rexp(c.h, ob.data_ptr(), act.data_ptr(), dt, buf.data_ptr(),
                                                  0 if k_shared else Bp * c.ldk, c.ldk, B, rexp.data_ptr(),
                                                  (c.L + 1) * Bp, Bp, c.L + 1, s), "amx_assemble_input_rexp")
        elif not assembled:  # (the device policy can write x0 itself: amx_policy_act's fused assembly)
            N.check(c.lib.amx_assemble_input(c.h, ob.data_ptr(), act.data_ptr(), dt, buf.data_ptr(), Bp * c.ldk,
                                             c.ldk, B, s), "amx_assemble_input")
        self._mlp(buf, preds, Bp, s, rexp, row_exponents=assembled, k_shared=k_shared)
        return preds

    def _mlp_h3(self, buf, preds, Bp, s, rexp, k_shared=0):
        c = self.ctx
        sA, sR, L = Bp * c.ldk, (c.L + 1) * Bp, c.L
        for i in range(L):
            K = c.k0_pad + i * c.Hp
            N.check(c.lib.amx_gemm_bias_act_h3(c.h, c.M, Bp, c.Hp, K, buf.data_ptr(), c.ldk, sA, self.W2[i].data_ptr(),
                                               c.Hp * 2 * K, self.wexp[i].data_ptr(), c.Hp, self.b[i].data_ptr(), c.Hp,
                                               buf.data_ptr(), c.ldk, sA, K, N.AMX_ACT_RELU, rexp.data_ptr(), sR,
                                               i + 1, rexp[0, i + 1].data_ptr(), k_shared, s), "amx_gemm_bias_act_h3")
        N.check(c.lib.amx_gemm_out_unnorm_h3(c.h, c.M, Bp, c.S, c.ldk, buf.data_ptr(), c.ldk, sA,
                                             self.W2[L].data_ptr(), c.n_out_pad * 2 * c.ldk, self.wexp[L].data_ptr(),
                                             c.n_out_pad, self.b[L].data_ptr(), c.n_out_pad, preds.data_ptr(), c.S,
                                             Bp * c.S, rexp.data_ptr(), sR, L + 1, k_shared, s),
                "amx_gemm_out_unnorm_h3")

    def _mlp(self, buf, preds, Bp, s, rexp, row_exponents=True, k_shared=0):
        c = self.ctx
        sA = Bp * c.ldk
        if self.W2 is not None and row_exponents:  # x0 row exponents (slot 0) + reset of the hidden slots
            N.check(c.lib.amx_row_exponents(c.h, c.M, Bp, c.k0_pad, buf.data_ptr(), c.ldk, sA, rexp.data_ptr(),
                                            (c.L + 1) * Bp, c.L + 1, s), "amx_row_exponents")
        ev = self.gemm_events
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if self.W2 is not None:
            self._mlp_h3(buf, preds, Bp, s, rexp, k_shared)
            if ev is not None:
                e1.record()
                ev.append((e0, e1, Bp))
            return
        for i in range(c.L):
            K = c.k0_pad + i * c.Hp
            if self.W3 is not None:
                N.check(c.lib.amx_gemm_bias_act_x6(c.h, c.M, Bp, c.Hp, K, buf.data_ptr(), c.ldk, sA,
                                                   self.W3[i].data_ptr(), c.Hp * 3 * K, self.b[i].data_ptr(), c.Hp,
                                                   buf.data_ptr(), c.ldk, sA, K, N.AMX_ACT_RELU, s),
                        "amx_gemm_bias_act_x6")
            else:
                N.check(c.lib.amx_gemm_bias_act(c.h, c.M, Bp, c.Hp, K, buf.data_ptr(), c.ldk, sA, self.W[i].data_ptr(),
                                                K, c.Hp * K, self.b[i].data_ptr(), c.Hp, buf.data_ptr(), c.ldk, sA,
                                                K, N.AMX_ACT_RELU, s), "amx_gemm_bias_act")
        if self.W3 is not None:
            N.check(c.lib.amx_gemm_out_unnorm_x6(c.h, c.M, Bp, c.S, c.ldk, buf.data_ptr(), c.ldk, sA,
                                                 self.W3[c.L].data_ptr(), c.n_out_pad * 3 * c.ldk,
                                                 self.b[c.L].data_ptr(), c.n_out_pad, preds.data_ptr(), c.S,
                                                 Bp * c.S, s), "amx_gemm_out_unnorm_x6")
        else:
            N.check(c.lib.amx_gemm_out_unnorm(c.h, c.M, Bp, c.S, c.ldk, buf.data_ptr(), c.ldk, sA,
                                              self.W[c.L].data_ptr(), c.ldk, c.n_out_pad * c.ldk,
                                              self.b[c.L].data_ptr(), c.n_out_pad, preds.data_ptr(), c.S, Bp * c.S, s),
                    "amx_gemm_out_unnorm")
        if ev is not None:
            e1.record()
            ev.append((e0, e1, Bp))

    def mlp_flops_per_sample(self) -> int:
        """Algorithmic FLOPs of one sample through all members (unpadded shapes)."""
        c, h = self.ctx, self.hidden
        macs = sum(h * (c.S + c.A + i * h) for i in range(c.L)) + c.S * (c.S + c.A + c.L * h)
        return 2 * macs * c.M

    def disagreement(self, preds: torch.Tensor, B: int, out: torch.Tensor | None = None) -> torch.Tensor:
        c = self.ctx
        out = torch.empty(B, dtype=torch.float32, device=c.device) if out is None else out
        N.check(c.lib.amx_disagreement(c.h, preds.data_ptr(), c.S, preds.shape[1] * c.S, out.data_ptr(), B, c.stream),
                "amx_disagreement")
        return out

    # ---- reference-compatible surface (milo/milo/dynamics.py) ------------------------------
    def get_action_discrepancy(self, state: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        """DynamicsEnsemble.get_action_discrepancy (dynamics.py:154-165): float32 inputs,
        returns the per-row max pairwise L2 disagreement [B] (on the device)."""
        state = state.to(self.ctx.device, torch.float32).contiguous()
        action = action.to(self.ctx.device, torch.float32).contiguous()
        if state.dim() == 1:
            state, action = state.unsqueeze(0), action.unsqueeze(0)
        B = state.shape[0]
        preds = self.forward_preds(state, action, B)
        return self.disagreement(preds, B)

    def compute_threshold(self, states: torch.Tensor, actions: torch.Tensor, batch: int = 65536) -> float:
        """compute_threshold (dynamics.py:145-152): max disagreement over the offline set."""
        best = None
        for i in range(0, states.shape[0], batch):
            d = self.get_action_discrepancy(states[i:i + batch], actions[i:i + batch]).max()
            best = d if best is None else torch.maximum(best, d)
        self.threshold = float(best.item())
        return self.threshold

    def model_forward(self, k: int, state: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        """models[k].forward(state, action, unnormalize_out=True) (dynamics.py:216-233)."""
        state = state.to(self.ctx.device, torch.float32).contiguous()
        action = action.to(self.ctx.device, torch.float32).contiguous()
        B = state.shape[0]
        return self.forward_preds(state, action, B)[k, :B].clone()


class RffMap:
    """phi(x) = cos(x W^T + b) * sqrt(2/F) on MFMA (linear_cost.py:64-71) with fp64 column sums."""

    def __init__(self, ctx: AmxContext, W: torch.Tensor, b: torch.Tensor, gemm: str = "f16x3"):
        """gemm: "f16x3" (amx_rff_features_h3 on the scaled 2-limb image of W), "bf16x6"
        (amx_rff_features_x6 on the 3-limb image) or "f32"."""
        if gemm not in DeviceEnsemble.GEMM_PRECISIONS:
            raise ValueError(f"gemm must be one of {DeviceEnsemble.GEMM_PRECISIONS}, got {gemm!r}")
        self.gemm = gemm
        self.ctx = ctx
        F, D = W.shape
        self.F, self.D = F, D
        self.Fp = round_up(F, 128)
        if self.Fp != F:
            raise ValueError("feature_dim must be a multiple of 128 for the MFMA RFF path")
        self.Kp = round_up(D, 32)
        Wp = torch.zeros(F, self.Kp, dtype=torch.float32)
        Wp[:, :D] = W.float().cpu()
        self.W = Wp.to(ctx.device).contiguous()
        self.b = b.float().to(ctx.device).contiguous()
        self.W3 = split_bf16x3(ctx, self.W.unsqueeze(0))[0] if gemm == "bf16x6" else None
        self.W2 = self.wexp = None
        if gemm == "f16x3":
            W2, wexp = split_f16x2(ctx, self.W.unsqueeze(0))
            self.W2, self.wexp = W2[0], wexp[0]
        # np.sqrt(2/F) is a float64 scalar; torch multiplies the fp32 tensor by it rounded to fp32
        self.scale = float(np.float32(np.sqrt(2 / F)))

    def features(self, x: torch.Tensor, rows: int, n_valid: int, phi: torch.Tensor, partials: torch.Tensor,
                 row_mask: torch.Tensor | None = None, ldx: int | None = None,
                 row_exp: torch.Tensor | None = None) -> None:
        """phi rows + fp64 column partials [rows / 32][F] (one per 32-row group, AMX_RFF_PART_ROWS)
        of x's `rows` rows.  f16x3: `row_exp` [rows] int32 = the rows' exponents (amx_step_rexp
        writes them for the rollout's [s, s'] rows); None computes them here (amx_row_exponents)."""
        c = self.ctx
        if partials.dtype != torch.float64 or partials.numel() < rows // N.RFF_PART_ROWS * self.F:
            raise ValueError(f"partials must be fp64 with room for [{rows // N.RFF_PART_ROWS}][{self.F}] "
                             f"(one row per {N.RFF_PART_ROWS} feature rows), got {tuple(partials.shape)} "
                             f"{partials.dtype}")
        ldx = self.Kp if ldx is None else ldx
        if self.W2 is not None:
            if row_exp is None:
                row_exp = torch.empty(rows, dtype=torch.int32, device=c.device)
                N.check(c.lib.amx_row_exponents(c.h, 1, rows, self.Kp, x.data_ptr(), ldx, 0, row_exp.data_ptr(), rows,
                                                1, c.stream), "amx_row_exponents")
            N.check(c.lib.amx_rff_features_h3(c.h, rows, n_valid, self.F, self.Kp, x.data_ptr(), ldx,
                                              self.W2.data_ptr(), self.wexp.data_ptr(), row_exp.data_ptr(),
                                              self.b.data_ptr(), self.scale, phi.data_ptr(), phi.shape[-1],
                                              partials.data_ptr(), None if row_mask is None else row_mask.data_ptr(),
                                              c.stream), "amx_rff_features_h3")
            return
        if self.W3 is not None:
            N.check(c.lib.amx_rff_features_x6(c.h, rows, n_valid, self.F, self.Kp, x.data_ptr(), ldx,
                                              self.W3.data_ptr(), self.b.data_ptr(), self.scale, phi.data_ptr(),
                                              phi.shape[-1], partials.data_ptr(),
                                              None if row_mask is None else row_mask.data_ptr(), c.stream),
                    "amx_rff_features_x6")
            return
        N.check(c.lib.amx_rff_features(c.h, rows, n_valid, self.F, self.Kp, x.data_ptr(), ldx, self.W.data_ptr(),
                                       self.Kp, self.b.data_ptr(), self.scale, phi.data_ptr(), phi.shape[-1],
                                       partials.data_ptr(), None if row_mask is None else row_mask.data_ptr(),
                                       c.stream), "amx_rff_features")

    def embed(self, x: torch.Tensor):
        """(phi [n, F], column sums [F] fp64) of arbitrary rows x [n, D] (fp32, any device)."""
        c = self.ctx
        n = x.shape[0]
        rows = round_up(max(n, 1), 128)
        # the 160 x 256 one-round tiles (amx_rff_features_h3) need rows = k * 160 * CUs / (F / 256):
        # worth ~1 % of padding rows (40 530 -> 40 960: 121 -> 76 us on 128 x 128 tiles)
        r160 = 160 * c.n_cus // max(self.F // 256, 1) if self.F % 256 == 0 else 0
        if self.W2 is not None and r160 and n >= r160 and round_up(n, r160) <= 1.05 * n:
            rows = round_up(n, r160)
        xp = torch.zeros(rows, self.Kp, dtype=torch.float32, device=c.device)
        xp[:n, :self.D] = x.to(c.device, torch.float32)
        phi = torch.empty(rows, self.F, dtype=torch.float32, device=c.device)
        part = torch.empty(rows // N.RFF_PART_ROWS, self.F, dtype=torch.float64, device=c.device)
        self.features(xp, rows, n, phi, part)
        tot = torch.empty(self.F, dtype=torch.float64, device=c.device)
        N.check(c.lib.amx_sum_partials(c.h, part.data_ptr(), rows // N.RFF_PART_ROWS, self.F, tot.data_ptr(), c.stream),
                "amx_sum_partials")
        return phi[:n], tot
