#!/usr/bin/env python
"""Headline benchmark: learned-dynamics env-steps/s of the full MILO rollout on MI355X.

Workload (BASELINE.json configs[2] at N=1, configs[3] at N>1): one bench step = one complete
40 000-sample MILO rollout, its lanes sharded over the N ranks (strong scaling; --samples-per-gpu
gives the weak-scaling form) — per rank B persistent humanoid3d lanes x T synchronous steps of {device Gaussian-MLP policy -> 4-model dense [512]x4 ensemble ->
fp64 state update + fall/horizon termination + disagreement -> RFF (s,s') features ->
auto-reset}, then the relabel {ordered fp64 feature sum -> RCCL all-reduce (N>1) -> MMD
witness -> per-sample pessimistic reward -> expert cost over the resident 50k-row expert
buffer}.  Synthetic data of the BASELINE shape (obs 197, act 36; --faithful for the
226/28 layout the reference scene actually builds) and random-init weights of the
reference architecture.  Inputs are resident in HBM before timing starts.

Launch: python bench.py [--gpus N --steps K --warmup W]; N>1 either via torch.distributed.run
(WORLD_SIZE set: it must equal --gpus) or directly, in which case bench.py starts the N rank
processes itself (one per GPU, RCCL).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (matrix), v_mfma_f32_32x32x2_f32
# bf16 dense MFMA: 256 CUs x 4 SIMDs x 1024 FLOP/clk (v_mfma_f32_32x32x16_bf16: 32 cycles) x 2.4 GHz
BF16_MFMA_PEAK_TFLOPS = 2516.6
# the bf16x6 GEMM issues 6 bf16 limb products per f32 multiply-add, the f16x3 GEMM 3 fp16 limb
# products (fp16 dense MFMA = the bf16 rate): their f32-equivalent ceilings
X6_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6
H3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3
GEMM_INFO = {
    "f16x3": dict(peak=H3_PEAK_TFLOPS, products=3,
                  desc="f16x3: fp32 operands scaled by powers of two (per weight row / activation row) and split "
                       "into 2 fp16 limbs, 3 limb products per f32 MAC accumulated in fp32 (error vs fp64 <= the "
                       "f32 MFMA's, tools/h3_accuracy.py)",
                  unit="TFLOP/s (f32-equivalent; peak = f16 dense 2516.6 / 3 limb products)",
                  kernel="k_gemm_h3 (ensemble layers: hidden and output layers on v_mfma_f32_16x16x32_f16; "
                         "3 per f32 MAC)",
                  dtype="fp32 (f16x3-emulated: 2 scaled fp16 limbs, 3 MFMA products per f32 MAC, fp32-level error)",
                  peak_note="frac is against the f16 matrix pipe's dense peak / 3 (838.9 TF/s f32-equivalent); "
                            "frac_vs_f32_mfma against the native FP32 MFMA peak (157.3 TF/s), which this "
                            "emulation exceeds"),
    "bf16x6": dict(peak=X6_PEAK_TFLOPS, products=6,
                   desc="bf16x6: fp32 operands split exactly into 3 bf16 limbs, 6 limb products per f32 MAC "
                        "accumulated in fp32 (error vs fp64 = the f32 MFMA's, tools/x6_accuracy.py)",
                   unit="TFLOP/s (f32-equivalent; peak = bf16 dense 2516.6 / 6 limb products)",
                   kernel="k_gemm_x6 (ensemble layers, v_mfma_f32_32x32x16_bf16 x 6 per f32 MAC)",
                   dtype="fp32 (bf16x6-emulated: 3 bf16 limbs, 6 MFMA products per f32 MAC, fp32-level error)",
                   peak_note="frac is against the bf16 matrix pipe's dense peak / 6 (419.4 TF/s f32-equivalent); "
                             "frac_vs_f32_mfma against the native FP32 MFMA peak (157.3 TF/s)"),
    "f32": dict(peak=F32_MFMA_PEAK_TFLOPS, products=None, desc="f32 MFMA (v_mfma_f32_32x32x2_f32)",
                unit="TFLOP/s", kernel="k_gemm_nt (ensemble layers, f32 MFMA 32x32x2)", dtype="fp32",
                peak_note="native FP32 MFMA peak"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20, help="timed rollouts")
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--total-samples", type=int, default=40000,
                   help="samples per rollout over ALL ranks (strong scaling: the 40 000-sample rollout sharded "
                        "across the GPUs, BASELINE configs[3]); default")
    p.add_argument("--samples-per-gpu", type=int, default=0,
                   help="weak scaling instead: this many samples per rollout on every rank")
    p.add_argument("--lanes", type=int, default=0, help="persistent env lanes per GPU (0: automatic)")
    p.add_argument("--max-lanes", type=int, default=8192)
    p.add_argument("--faithful", action="store_true", help="use the 226/28 state/action layout")
    p.add_argument("--cost", choices=["mmd", "gail", "amp"], default="mmd",
                   help="amp: LS discriminator on AMP pose features of (s, s') with reference-motion resets "
                        "(BASELINE configs[4]; implies --faithful)")
    p.add_argument("--gemm", choices=["f16x3", "bf16x6", "f32"], default="f16x3",
                   help="ensemble GEMM: scaled 2-limb fp16 split (3 products) or 3-limb bf16 split (6 products) on "
                        "the 16-bit MFMA pipe (both fp32-level error), or f32 MFMA")
    p.add_argument("--expert-rows", type=int, default=50000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-workers", type=int, default=0)
    p.add_argument("--cpu-samples", type=int, default=0,
                   help="env-steps per worker at each sweep point (default: sized for --cpu-point-s)")
    p.add_argument("--cpu-point-s", type=float, default=3.0, help="seconds of sampling per sweep point")
    p.add_argument("--cpu-final-samples", type=int, default=120000,
                   help="env-steps of each of the three timed best-W runs (three 40 000-sample rollouts: ~8-12 s "
                        "of CPU work per run on a 16-core share)")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL on ROCm) or gloo (rehearsal)")
    p.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                   help="replay the whole rollout as captured HIP graph(s); auto = off: eager launches measured "
                        "faster at every per-rank share on ROCm 7 (profiles/r05z_graph_vs_eager.txt)")
    p.add_argument("--score-overlap", choices=["on", "off"], default="off",
                   help="score each step's cost rows on a side stream under the next step's policy "
                        "(RolloutEngine.score_overlap; bit-identical to the batched pass at the rollout's end; measured "
                        "1.6 %% slower at 8192 x 5, profiles/r06h_score_overlap_ab.txt)")
    p.add_argument("--fuse-assembly", choices=["on", "off"], default="off",
                   help="f16x3: the policy launch also writes the ensemble's x0 slice (RolloutEngine.fuse_assembly)")
    p.add_argument("--overlap", choices=["on", "off"], default="off",
                   help="N > 1: overlap each rollout's all-reduce with the next rollout's first forward (valid "
                        "only while consecutive rollouts share the policy: fixed-policy collection / evaluation; "
                        "a trainer updates the policy between iterations, so the default is the serial order)")
    p.add_argument("--paths-serial", action="store_true",
                   help="--mode paths: the serial chunk loop (read each chunk's done flags before queueing the next)")
    p.add_argument("--paths-chunk", type=int, default=16,
                   help="--mode paths: synchronous steps per sampler chunk (one host round trip each)")
    p.add_argument("--mode", choices=["engine", "paths", "train"], default="engine",
                   help="engine: persistent lanes x synchronous steps + device relabel (throughput); paths: the "
                        "reference's semantics through the drop-in surfaces -- sample_points(num_to_collect, "
                        "num_workers=--workers): complete exact-seeded trajectories per worker quota, path dicts "
                        "on the host -- then relabel_paths (batch_reinforce.py:88-169); train: the engine rollout + "
                        "relabel followed by the learner half of BatchREINFORCE.train_step on the device -- MLP "
                        "baseline values, GAE, whitening and the NPG update (10-step CG, kl_dist 0.05) with the "
                        "sampler's policy refreshed (batch_reinforce.py:170-200, npg_cg.py:113-199); the baseline's "
                        "Adam fit stays with the caller and is not timed; one rank")
    p.add_argument("--workers", type=int, default=4, help="--mode paths: sampler workers (run.py --num_cpu, default 4)")
    p.add_argument("--motion", default=None, help="--cost amp: character + clip bundle (tools/pack_motion.py)")
    p.add_argument("--dry-run", action="store_true",
                   help="print this rank's launch layout (rank, world, rendezvous) and exit before any GPU or "
                        "CPU-baseline work (checks the --gpus N process launch)")
    p.add_argument("--dry-run-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    p.add_argument("--dry-run-hang-rank", type=int, default=-1,
                   help="--dry-run at N > 1: the ranks join one CPU (gloo) all-reduce, except this one, which "
                        "sleeps (checks that a hung collective ends the run at --dist-timeout)")
    p.add_argument("--dist-timeout", type=float, default=300.0,
                   help="seconds a rendezvous or collective may block before the rank exits non-zero (the process "
                        "group's timeout; RCCL's watchdog tears the process down, TORCH_NCCL_ASYNC_ERROR_HANDLING=1)")
    p.add_argument("--diag-rollouts", type=int, default=5,
                   help="N > 1: untimed rollouts after the timed region with the all-reduce bracketed by HIP events "
                        "(the line's dist_diag.allreduce_wait_us)")
    return p.parse_args()


def init_dist(backend: str, timeout_s: float, dev=None) -> None:
    """One process group per run, fail-fast: a rendezvous or collective that blocks longer than
    timeout_s raises (gloo) or is aborted by the RCCL watchdog, which tears the process down
    (async error handling 1), so a hung rank exits non-zero and launch_ranks stops the others."""
    import datetime
    import torch.distributed as dist
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = dict(timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kw["device_id"] = dev
    dist.init_process_group(backend, **kw)


def cpu_share() -> int:
    """CPUs this process may actually use: the affinity mask, the cgroup quota and the
    OMP_NUM_THREADS share the GPU box sets (os.cpu_count() shows the whole machine)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline_leg(S, A, args):
    """The oracle's restated reference sampler + host relabel, timed on this host's cores
    (BASELINE.md §3).  A W = 1 calibration point sets the sweep's sample sizes so that every
    sweep point (W = powers of two up to the CPU share this process has, plus the share
    itself) runs about --cpu-point-s seconds of sampling; the best W is then timed end to end
    (sampler + relabel, the relabel on the whole CPU share as the reference's one-process torch
    relabel would use it) on --cpu-final-samples env-steps, after one discarded warm-up run three
    times, the relabel on the same fixed sample each time: the value is the median run and all
    three are reported.  Runs before anything touches the GPU (the pools fork)."""
    from oracle import cpu_baseline as cb
    share = cpu_share()
    if args.cpu_workers:
        grid = [args.cpu_workers]
    else:
        grid = sorted({w for w in (1, 2, 4, 8, 16, 32, 64, 128, 256) if w <= share} | {share})
    cal = cb.run(S, A, workers=1, samples=300, expert_rows=args.expert_rows, relabel=False)
    rate1 = cal["sampler_steps_per_s"]
    sweep = []
    for w in grid:
        n = args.cpu_samples * w if args.cpu_samples else int(max(300 * w, args.cpu_point_s * rate1 * w))
        r = cb.run(S, A, workers=w, samples=n, expert_rows=args.expert_rows, relabel=False)
        sweep.append((w, r))
    best_w, best = max(sweep, key=lambda x: x[1]["sampler_steps_per_s"])
    # one discarded warm-up end-to-end run (it also keeps the fixed relabel sample: a cold host
    # runs its first all-core pass at a higher boost clock, 10-20 % above the runs after it on
    # the round-4 boxes), then three end-to-end runs at the best W, sampler and relabel
    # interleaved; every run's sampler draws the same seeded trajectories and every relabel runs
    # on the SAME fixed sample, so the runs differ only by the host's timing noise; the value is
    # the median run
    n_final = max(best["samples"], args.cpu_final_samples)
    warm = cb.run(S, A, workers=best_w, samples=n_final, expert_rows=args.expert_rows, relabel=False, keep_paths=True)
    paths = warm.pop("_paths")
    warm_rel = cb.relabel_seconds(paths, S, A, expert_rows=args.expert_rows, threads=share)
    samp, rel = [], []
    for _ in range(3):
        samp.append(cb.run(S, A, workers=best_w, samples=n_final, expert_rows=args.expert_rows, relabel=False))
        rel.append(cb.relabel_seconds(paths, S, A, expert_rows=args.expert_rows, threads=share))
    finals = [dict(r, relabel_s=t, relabel_threads=share, end_to_end_steps_per_s=r["samples"] / (r["sampler_s"] + t))
              for r, t in zip(samp, rel)]
    best = sorted(finals, key=lambda r: r["end_to_end_steps_per_s"])[1]
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    pts = ", ".join(f"W={w}: {r['sampler_steps_per_s']:.0f} ({r['sampler_s']:.1f}s)" for w, r in sweep)
    e2e = [round(r["end_to_end_steps_per_s"], 1) for r in finals]
    return {
        "value": round(best["end_to_end_steps_per_s"], 1), "unit": "env-steps/s", "cores": best["workers"],
        "kind": "port",
        "sample": (f"{best['samples']} env-steps ({best['paths']} complete trajectories) by {best['workers']} "
                   f"forked sampler workers (torch threads 1) + host relabel (fit_cost + per-path bonus costs, "
                   f"{args.expert_rows}-row expert buffer, {best['relabel_threads']} torch threads); sampler alone "
                   f"{best['sampler_steps_per_s']:.0f} env-steps/s; sampler {best['sampler_s']:.2f}s + relabel "
                   f"{best['relabel_s']:.2f}s; median of 3 end-to-end runs after a discarded warm-up run (the "
                   f"relabel timed on the same fixed sample each time)"),
        "warmup_run": round(warm["samples"] / (warm["sampler_s"] + warm_rel), 1),
        "end_to_end_runs": e2e,
        "sampler_s_runs": [round(r["sampler_s"], 3) for r in finals],
        "relabel_s_runs": [round(r["relabel_s"], 3) for r in finals],
        "spread": round((max(e2e) - min(e2e)) / max(e2e), 4),
        "sweep_sampler_steps_per_s": pts,
        "best_workers": best_w, "relabel_threads": best["relabel_threads"],
        "cpu_share": share, "os_cpu_count": os.cpu_count(), "cpu_model": cpu,
    }


def gemm_source_sha16() -> str:
    """Hash of the GEMM kernel sources (csrc/amx_gemm.hip + amx_h3.h): the key that ties a PMC
    traffic record to the build it was measured on."""
    import hashlib
    h = hashlib.sha256()
    for name in ("amx_gemm.hip", "amx_h3.h"):
        with open(os.path.join(ROOT, "amp_extensions_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def gemm_traffic(gemm: str, S: int, B: int):
    """(HBM bytes per ensemble-GEMM launch, note) from the PMC record that ships with the package
    (amp_extensions_amd/data/gemm_traffic_<gemm>.json, written by tools/pmc_traffic.sh: FETCH_SIZE
    x 2 + WRITE_SIZE in separate rocprofv3 passes, MI355X_MICROARCH.md's gfx950 correction).  Only
    a record of THIS build's GEMM sources at this shape counts; otherwise traffic is null."""
    path = os.path.join(ROOT, "amp_extensions_amd", "data", f"gemm_traffic_{gemm}.json")
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, f"no PMC record ({os.path.relpath(path, ROOT)})"
    if tj.get("state_dim") != S or tj.get("lanes") != B or tj.get("gemm", "f32") != gemm:
        return None, f"PMC record is for S={tj.get('state_dim')} lanes={tj.get('lanes')} gemm={tj.get('gemm')}"
    if tj.get("gemm_source_sha16") != gemm_source_sha16():
        return None, "PMC record is from another build of the GEMM sources"
    return tj.get("hbm_bytes_per_launch"), (
        f"rocprofv3 PMC, (2*FETCH_SIZE + WRITE_SIZE) per launch averaged over the forward's layers; "
        f"{tj.get('ratio')}x the algorithmic {tj.get('alg_bytes_per_launch')} B; build {tj.get('gemm_source_sha16')}")


def plan_lanes(samples: int, max_lanes: int, lanes: int = 0):
    """(lanes, sync steps) of one rank's rollout.  Lane counts are multiples of 1024 in
    [4096, max_lanes]: with 4 members they give the ensemble GEMMs one full 256-workgroup wave
    (256 x 256 tiles at 8192 lanes, the row-block tiles RB x 256 at 32 RB lanes otherwise).
    Among the step counts T = ceil(samples / max_lanes) and T + 1 the one with the smaller
    modelled time T * (60 us + 53 ns * lanes) wins (per-step fixed cost + per-lane GEMM cost,
    measured at 8192 lanes)."""
    if lanes:
        return lanes, math.ceil(samples / lanes)
    best = None
    T0 = max(1, math.ceil(samples / max_lanes))
    for T in (T0, T0 + 1):
        L = min(max_lanes, max(4096, (math.ceil(samples / T) + 1023) // 1024 * 1024))
        t = T * (60e-6 + 53e-9 * L)
        if L * T >= samples and (best is None or t < best[0]):
            best = (t, L, T)
    return best[1], best[2]


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N fresh rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1),
    as the reference's sampler starts its worker pool inside the call
    (milo/milo/sampler.py:111-121).  The parent never touches the GPU (no torch import, no HIP
    call: the children are plain child processes, nothing is exec'ed over a GPU process); rank
    0 prints the JSON line.  Returns the worst exit status."""
    import signal
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))

    def forward(sig, _frame):  # a launcher/timeout signalling the parent reaches the ranks too
        for q in procs:
            if q.poll() is None:
                q.send_signal(sig)
        raise SystemExit(128 + sig)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    try:
        while [p.poll() for p in procs].count(None):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad and rc == 0:
                rc = bad[0]
                for q in procs:  # one rank failed: the others would wait in a collective forever
                    if q.poll() is None:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
        if rc == 0:
            rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def main():
    args = parse()
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}")
    elif args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        print(json.dumps({"rank": rank, "local_rank": local, "world": world, "pid": os.getpid(),
                          "master": f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}"}),
              flush=True)
        if rank == args.dry_run_fail_rank:
            raise SystemExit(3)
        if args.dry_run_fail_rank >= 0:
            time.sleep(60)  # the launcher must stop the surviving ranks
        if args.dry_run_hang_rank >= 0 and world > 1:
            import torch
            import torch.distributed as dist
            init_dist("gloo", args.dist_timeout)
            if rank == args.dry_run_hang_rank:
                time.sleep(120)  # never joins: the others' all-reduce must time out
            dist.all_reduce(torch.ones(4))
            dist.destroy_process_group()
        return
    if args.cost == "amp":
        args.faithful = True   # the AMP features are defined on the humanoid3d CtController state
    S, A = (226, 28) if args.faithful else (197, 36)

    cpu_base = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        cpu_base = cpu_baseline_leg(S, A, args)

    import numpy as np
    import torch
    import torch.distributed as dist

    import amp_extensions_amd as amx
    from amp_extensions_amd import synthetic as syn
    from amp_extensions_amd.policy import init_mlp_policy_params

    # one rank per GPU; (local % device_count) only matters for a gloo rehearsal of several
    # ranks on one card
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        init_dist(args.dist_backend, args.dist_timeout, dev)
    # the fused [sum phi, count] all-reduce; after the timed region (dist_diag) its calls are
    # bracketed by HIP events on the current stream: the wait for the collective, including the
    # slowest rank's arrival
    ar_diag = {"on": False, "ev": []}

    def _allreduce(t):
        if not ar_diag["on"]:
            return dist.all_reduce(t)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dist.all_reduce(t)
        e1.record()
        ar_diag["ev"].append((e0, e1))
    allreduce = _allreduce if world > 1 else None
    # the overlapped form: the all-reduce is queued asynchronously (GPU-side wait) and runs under
    # the next rollout's first ensemble forward (RolloutEngine.rollout_overlapped)
    allreduce_async = (lambda t: dist.all_reduce(t, async_op=True)) if world > 1 else None

    # ---- model + data setup (untimed) -------------------------------------------------------
    hidden = [512] * 4
    M = 4
    s, a, s2 = syn.offline(100000, S, A, 0)
    st, at, s2t = (torch.from_numpy(x).float() for x in (s, a, s2))
    from amp_extensions_amd.datasets import get_transformations
    norms = get_transformations(st, at, s2t)
    from amp_extensions_amd.ensemble import init_ensemble_weights
    ens_w = init_ensemble_weights(S, A, hidden, M, base_seed=100)
    ctx = amx.AmxContext(S, A, n_models=M, hidden=512, n_hidden=4, feat_dim=512, device=dev)
    ens = amx.DeviceEnsemble(ctx, ens_w, norms, gemm=args.gemm)
    thr = ens.compute_threshold(st.to(dev), at.to(dev))
    reset_source = syn.reset_table(65536, S, 1)
    if args.cost == "amp":
        # humanoid3d + spinkick clip (the package's data bundle, amp_extensions_amd/data, or --motion);
        # expert rows = AMP features of the clip at uniform times (RecordAMPObsExpert)
        from amp_extensions_amd.motion import ReferenceMotion
        reset_source = ReferenceMotion.from_bundle(ctx, args.motion)
        times = np.random.RandomState(3).uniform(1.0 / 30, reset_source.get_motion_length(), args.expert_rows)
        expert = reset_source.expert_amp_obs(times).float().cpu()
    else:
        expert = torch.from_numpy(syn.expert(args.expert_rows, S, 3))
    if args.cost == "mmd":
        cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, bw_samples=100000, lambda_b=0.0025,
                                 seed=100, ctx=ctx)
    elif args.cost == "gail":
        cost = amx.GAILCost(expert, hidden_dims=(1024, 512), lambda_b=0.0025, seed=100, ctx=ctx)
    else:
        cost = amx.GAILCost(expert, hidden_dims=(1024, 512), input_type="amp", lambda_b=0.0025, seed=100, ctx=ctx,
                            motion=reset_source)
    pw, log_std = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=1000 + rank)
    strong = not args.samples_per_gpu
    per_rank = math.ceil(args.total_samples / world) if strong else args.samples_per_gpu
    B, T = plan_lanes(per_rank, args.max_lanes, args.lanes)
    eng = amx.RolloutEngine(ens, reset_source, lanes=B, policy=pol, cost=cost,
                            seed=(7 << 32) + rank, max_steps=T)
    eng.fuse_assembly = args.fuse_assembly == "on"
    eng.score_overlap = args.score_overlap == "on"
    eng.reset_all()
    # steady-state phase: a long-running lane fleet has its trajectories at uniformly spread
    # positions, so horizon resets (1/300 per step) happen inside the timed region as they do
    # in the reference's sampler; a fresh reset_all would put every lane at step 0
    horizon = eng.term.horizon
    eng.num_steps.copy_(torch.randint(0, horizon, (B,), generator=torch.Generator().manual_seed(11 + rank),
                                      dtype=torch.int32).to(dev))

    # N > 1 (MMD): each rank scores N_e / N expert rows in its relabel and the fp64 partial sums
    # are all-reduced asynchronously (the expert cost is the bonus_mmd log's term),
    # waited for (GPU-side) only before the next relabel overwrites the sum
    shard = world > 1 and args.cost == "mmd" and args.mode == "engine"
    if shard:
        cost.shard_expert(rank, world, allreduce_async)

    def one_rollout():
        eng.rollout(T)
        eng.relabel(allreduce)  # MMD: feature mean -> w -> rewards (GAIL: rewards already scored)
        if shard:
            cost.expert_allreduce()
        elif args.cost == "mmd":
            cost.get_expert_cost()
        return T * B

    paths_info = {}
    if args.mode == "train":
        # MILO's learner settings (milo/milo/arguments.py:100-122): critic [128, 128], gamma 0.995,
        # gae_lambda 0.97, cg_iter 10, cg_damping 1e-4, kl_dist 0.05, hvp_sample_frac 1
        if world > 1:
            raise SystemExit("bench.py --mode train: one rank (the device NPG reduces over one process's samples)")
        from amp_extensions_amd.gae import init_mlp_baseline_params
        baseline = amx.DeviceMLPBaseline(ctx, init_mlp_baseline_params(S, (128, 128), seed=7))
        npg = amx.DeviceNPG(ctx, pw, log_std, kl_dist=0.05, FIM_invert_args={"iters": 10, "damping": 1e-4},
                            policy=pol)

        def one_rollout():
            eng.rollout(T)
            eng.relabel(allreduce)
            if args.cost == "mmd":
                cost.get_expert_cost()
            adv = eng.advantages(baseline, gamma=0.995, gae_lambda=0.97)["advantages"]
            info = npg.train_from_engine(eng, adv)
            paths_info.update(kl=info["kl_dist"], alpha=info["alpha"])
            return T * B

    if args.mode == "paths":
        # the reference's call sequence (batch_reinforce.py:88-90, 103-169): sample_points with W
        # workers' exact-seeded trajectories (path dicts on the host), then the relabel of those
        # paths; this rank's workers get their own seed block
        from amp_extensions_amd.relabel import relabel_paths
        it = [0]

        def one_rollout():
            it[0] += 1
            paths = amx.sample_points(eng, pol, num_to_collect=per_rank, base_seed=1000 * rank + it[0],
                                      num_workers=args.workers, chunk=args.paths_chunk,
                                      pipeline=not args.paths_serial)
            relabel_paths(paths, cost, ens, allreduce=allreduce)
            n = sum(len(p["rewards"]) for p in paths)
            paths_info.update(paths=len(paths), samples=n)
            return n

    # the in-kernel GEMM timer is registered before the warm-up: graphs captured there (the
    # sampler's chunk graphs in paths mode) carry its buffer in their GEMM arguments, so their
    # replays in the timed region are timed too (it is zeroed before the timed region)
    timer = ctx.gemm_timer() if args.gemm == "f16x3" else None
    for _ in range(args.warmup):
        one_rollout()
    torch.cuda.synchronize()

    # HIP graph: the whole rollout (steps, scoring, relabel, expert cost) is captured once and
    # replayed, so per-kernel host launch overhead leaves the timed region (the RCCL all-reduce
    # of N>1 runs eagerly between two graphs).  The f16x3 ensemble GEMMs time themselves in
    # both launch modes (amx_set_gemm_timer: start stamp in the first layer, tick sum in the
    # output layer's last workgroup; no extra launches): ROCm has no timing-event nodes in
    # graphs, and in eager mode each timing-event record is a queue drain that opened a
    # 5.6 us gap before the first and after the last GEMM of every step (rocprofv3 trace,
    # profiles/r02_event_gaps.txt) -- 2 % of the timed region.  The other GEMM paths keep
    # HIP events.
    # (auto: eager.  Round 2 replayed small per-rank rollouts as graphs to hide the host launch
    # cost; on the round-5 kernels eager launches are 1.6-1.9 % faster at the N = 4 / 8 shares and
    # 1 % at N = 1, profiles/r05z_graph_vs_eager.txt: the host stays ahead of the GPU either way.)
    graph = None
    use_graph = args.mode == "engine" and args.graph == "on"
    if use_graph and args.gemm != "f16x3":
        raise SystemExit("--graph needs the f16x3 GEMM (its in-kernel timer)")
    # --overlap on (N > 1, MMD): each rollout's all-reduce overlaps the next rollout's first
    # forward and its relabel runs after that forward; the last relabel is flushed inside the
    # timed region (the first timed rollout also recomputes the warm-up's relabel: one extra
    # relabel timed).  Off by default: a trainer's policy update sits between two iterations'
    # rollouts, so the headline keeps the serial rollout -> all-reduce -> relabel order.
    overlap = world > 1 and args.cost == "mmd" and args.overlap == "on"
    tail = cost.get_expert_cost if args.cost == "mmd" and not shard else None
    hooks = dict(before_relabel=cost.wait_expert_allreduce, after=cost.expert_allreduce_replayed) if shard else {}
    flush = eng.flush_relabel
    if use_graph:
        if overlap:
            graph, flush = eng.graph_rollout_overlapped(T, allreduce_async, tail=tail, **hooks)
            graph()  # warm replay
            flush()
        else:
            graph = eng.graph_rollout(T, allreduce=allreduce, tail=tail, **hooks)
            graph()  # warm replay
    torch.cuda.synchronize()
    if timer is not None:
        timer.zero_()

    # ---- timed region -----------------------------------------------------------------------
    ens.gemm_events = [] if timer is None else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    samples = 0
    if graph is None and overlap:
        for _ in range(args.steps):
            samples += eng.rollout_overlapped(T, allreduce_async, tail=cost.expert_allreduce if shard else tail)
        flush()
    elif graph is None:
        for _ in range(args.steps):
            samples += one_rollout()
    else:
        for i in range(args.steps):
            samples += graph()
        if overlap:
            flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    term_rate = float(eng.done[:T].float().mean().item()) if args.mode != "paths" else None
    own_elapsed = elapsed
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    total_samples = samples * world

    # dominant kernel: the ensemble GEMM launches (HIP events on the launch stream)
    if timer is None:
        gemm_ms = sum(e0.elapsed_time(e1) for (e0, e1, _) in ens.gemm_events)
        n_fwd = len(ens.gemm_events)
    else:
        tv = timer.cpu().numpy()
        gemm_ms = float(tv[2]) / 1e5  # 100 MHz ticks -> ms
        n_fwd = int(tv[3])
        ctx.gemm_timer(False)
    shard_note = (f"; expert cost over {args.expert_rows}/{world} expert rows per rank, its fp64 sum all-reduced "
                  f"off the critical path" if shard else "")
    per_fwd = ctx.L + 1  # GEMM launches per forward
    launches = n_fwd * per_fwd
    flops_per_fwd = ens.mlp_flops_per_sample() * B
    if args.mode == "paths":
        # the sampler's forwards run at its own lane counts (chunks of idle-padded lanes): count
        # the algorithmic FLOPs of the samples it returned over the forwards' measured time --
        # one member per sample while sampling (member-blocked lanes: SimEnv.step's one model;
        # every member without blocking) plus every member in the relabel's disagreement
        sampling = 1.0 / ctx.M if (args.gemm == "f16x3" and ctx.M >= 2) else 1.0
        flops_per_fwd = ens.mlp_flops_per_sample() * samples * (sampling + 1.0) / max(n_fwd, 1)
    achieved_tflops = flops_per_fwd * n_fwd / (gemm_ms * 1e-3) / 1e12
    ens.gemm_events = None

    # N > 1 diagnostics (untimed, after the timed region): the all-reduce wait per rollout, the
    # ranks' elapsed-time spread and every rank's GEMM fraction, gathered to rank 0
    dist_diag = None
    if world > 1:
        wait_us = float("nan")
        if args.diag_rollouts > 0 and args.mode == "engine" and not overlap:
            ar_diag["on"] = True
            for _ in range(args.diag_rollouts):
                one_rollout() if graph is None else graph()
            torch.cuda.synchronize()
            ar_diag["on"] = False
            if ar_diag["ev"]:
                wait_us = 1e3 * sum(a.elapsed_time(b) for a, b in ar_diag["ev"]) / len(ar_diag["ev"])
        mine = torch.tensor([own_elapsed, achieved_tflops / GEMM_INFO[args.gemm]["peak"], wait_us],
                            dtype=torch.float64, device=dev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        every = torch.stack(every).cpu().numpy()
        el = every[:, 0]
        dist_diag = {
            "world_size": dist.get_world_size(), "backend": args.dist_backend,
            "elapsed_s_per_rank": [round(float(x), 6) for x in el],
            "elapsed_spread": round(float((el.max() - el.min()) / el.max()), 4),
            "gemm_frac_per_rank": [round(float(x), 4) for x in every[:, 1]],
            "allreduce_wait_us_per_rank": [None if np.isnan(x) else round(float(x), 1) for x in every[:, 2]],
            "allreduce_note": (f"HIP events around the fused [sum phi, count] all-reduce on the current stream over "
                               f"{args.diag_rollouts} untimed rollouts after the timed region (includes waiting for "
                               f"the slowest rank)"),
            "dist_timeout_s": args.dist_timeout,
        }

    # + the cost's share: RFF features, or the discriminator MLP on its input
    if args.cost == "mmd":
        step_flops = ens.mlp_flops_per_sample() + 2 * (2 * S) * 512
    else:
        step_flops = ens.mlp_flops_per_sample() + 2 * (cost.input_dim * 1024 + 1024 * 512 + 512)
    value = total_samples / elapsed
    if args.mode == "paths":
        # the sampler's forwards run at its own (chunk-dependent) lane counts, which no PMC record covers
        traffic, traffic_note = None, "paths mode: the sampler's forwards run at other lane counts than the PMC record's"
    else:
        traffic, traffic_note = gemm_traffic(args.gemm, S, B)

    gi = GEMM_INFO[args.gemm]
    peak = gi["peak"]
    if rank == 0:
        out = {
            "metric": "learned-dynamics env steps/sec (humanoid3d, 40k-sample rollout)",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": gi["dtype"],
            "data": "synthetic (SURVEY §8d distributions; random-init reference architecture)",
            "config": {
                "workload": "full MILO rollout: policy + 4-model ensemble step + termination + " + {
                    "mmd": "RFF-MMD relabel",
                    "gail": "AMP/GAIL LS-disc reward on [s, s']",
                    "amp": "AMP LS-disc reward on AMP pose features of (s, s'), reference-motion resets"}[args.cost],
                "samples_per_rollout": T * B * world, "samples_per_rollout_per_gpu": T * B,
                "lanes_per_gpu": B, "sync_steps": T,
                "launch": "eager" if graph is None else "HIP graph replay of the whole rollout",
                **({} if args.mode != "train" else {
                    "mode": ("train: rollout + relabel + MLP-baseline values + GAE + whitening + NPG update "
                             "(VPG, 10-step CG on the Fisher, step, surrogate/KL) + policy refresh per step, all on "
                             "the device; the baseline's Adam fit is the caller's and is not timed"),
                    "npg_kl_last": round(float(paths_info.get("kl", 0.0)), 5)}),
                **({} if args.mode != "paths" else {
                    "mode": (f"reference semantics: sample_points(num_to_collect={per_rank}, num_workers="
                             f"{args.workers}) -> complete exact-seeded trajectories (per-worker quota "
                             f"ceil(N/W)), host path dicts -> relabel_paths; chunks of {args.paths_chunk} steps replayed as "
                             f"HIP graphs, speculative admission"),
                    "samples_per_rollout": paths_info.get("samples", 0) * world,
                    "samples_per_rollout_per_gpu": paths_info.get("samples", 0),
                    "paths_per_rollout_per_gpu": paths_info.get("paths", 0),
                    "lanes_per_gpu": None, "sync_steps": None, "launch": "sampler chunks"}),
                "state_dim": S, "action_dim": A, "ensemble": "4 x dense-connect [512]x4 ReLU",
                "rff_features": 512, "expert_rows": args.expert_rows, "policy": "tanh MLP(32,32)",
                "parallelism": (f"dp{world} (the {args.total_samples}-sample rollout's lanes sharded over the "
                                f"ranks, 1 all-reduce of [sum phi, count] per rollout"
                                f"{shard_note}"
                                f"{', overlapped with the next rollout' + chr(39) + 's first forward' if overlap else ''})"
                                if strong else
                                f"dp{world} (lane-sharded, {args.samples_per_gpu} samples per rank, 1 all-reduce "
                                f"per rollout)"),
                "termination_rate": None if term_rate is None else round(term_rate, 5), "threshold": thr,
                "gemm": gi["desc"],
            },
            "roofline": {
                "bound": "mfma", "achieved": round(achieved_tflops, 2), "peak": round(peak, 1),
                "unit": gi["unit"],
                "frac": round(achieved_tflops / peak, 4), "traffic": traffic, "traffic_note": traffic_note,
                "frac_vs_f32_mfma": round(achieved_tflops / F32_MFMA_PEAK_TFLOPS, 4),
                "peak_note": gi["peak_note"],
                "kernel": gi["kernel"],
                "matrix_pipe_tflops": round(gi["products"] * achieved_tflops, 1) if gi["products"] else None,
                "avg_launch_us": round(gemm_ms * 1e3 / max(launches, 1), 2),
                "timing": ("HIP events around the GEMM launches" if timer is None else
                           "in-kernel device realtime (amx_set_gemm_timer, 100 MHz, on the launch stream): first "
                           "hidden layer's start to the output layer's last workgroup, per forward (event records "
                           "drain the queue: 5.6 us gaps; no timing events in graphs)"),
                "flops_per_launch": flops_per_fwd / per_fwd,
            },
            "step_flops_frac": round(value / world * step_flops / (peak * 1e12), 4),
            "cpu_baseline": cpu_base,
            **({} if dist_diag is None else {"dist_diag": dist_diag}),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
