"""Benchmark: CIFAR-10 forward-invariance (Lyapunov) train step, images/sec, on 1..N MI355X.

python bench.py --gpus N --steps K --warmup W           (N>1: launched by torch.distributed.run)

One step (per rank, B=128 images, h_sample_size S=256 at epoch 20: S1=204 Uniform + S2=52
CorrectCone rows per image, N=32,768 rows) = the reference's training_step + backward + Adam:
  backbone KWLarge-Cayley (PyTorch-ROCm)  ->  Cayley maps of the 4 dynamics layers  ->
  fused HIP fan-out step (libfiode.so: sampler, 2 eval_dot passes incl. the bisection QP with the
  batch-global exit, V / V-dot, hinge loss, logging statistics, all dynamics gradients)  ->
  autograd through Cayley + backbone  ->  [RCCL all-reduce of the flat gradient + the fused
  metric scalars]  ->  Adam.
Inputs are synthetic (x ~ U[0,1), y ~ randint(10), seeded), resident in HBM before timing.

Besides the JSON fields of the contract, the line carries:
  roofline      the dominant fused kernel's algorithmic FLOP / its mean duration (HIP events
                recorded by libfiode on the kernels' stream) vs the f32 MFMA peak
  cpu_baseline  the same step on the host cores (backbone + Cayley maps + the reference fan-out
                restated op for op in torch, oracle/torch_ref.py, + train_ode + Adam), median of
                up to 20 steps after 3 warm-ups within a bounded budget, rank 0 at N=1 only
  hot_path      images/sec of the fused kernels alone (no backbone / optimizer)
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
for _p in (ROOT, ROOT / "fi-ode_amd"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "CIFAR-10 train-step images/sec (B=128, h_sample=256) at 1/2/4/8 MI355X"
B_PER_RANK = 128
H_SAMPLE = 256
EPOCH = 20
TRAIN_ODE_EPOCH = 10          # train_ode branch active at EPOCH (loss_ode portion 0.2)
MFMA_F32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: dense f32 MFMA (= f32 vector) peak
HBM_PEAK_GBS = 8000.0
# algorithmic FLOP per (image, sample) row
FLOP_ROW_FWD_PASS = 2 * (10 * 128 + 128 * 128 + 128 * 10)          # 37,888 per eval_dot pass
FLOP_ROW = {"k_lyap_fwd": 2 * FLOP_ROW_FWD_PASS,                   # loss pass + logging pass
            # input grads dL/da2 -> dL/da1 + weight grads dQ3, dQ2, dQ1 (the fused backward's
            # recompute of layers 1-2 is not algorithmic work and is not counted)
            "k_lyap_bwd": 2 * (128 * 128 + 128 * 10) + FLOP_ROW_FWD_PASS}


def build_module(dev, seed=0, train_ode=False, solver="rk4", h_sample=H_SAMPLE):
    from fiode_amd.dynamics import OrthoClassDynProjectSimplexLips
    from fiode_amd.lyapunov import LyapunovLearning, UniformInitFun, DecisionBoundary
    from fiode_amd.models import make_ortho_KWLarge_Concat
    from fiode_amd.sampling import (CompositeSampler, CompositeSamplerScheduler, CorrectConeSampling,
                                    LinearScheduler, UniformSimplexSampling)
    torch.manual_seed(seed)
    # README.md:27 over configs/classification/cifar_train.yaml
    dyn = OrthoClassDynProjectSimplexLips(n_hidden=10, activation="ReLU", dropout=0.5, mlp_size=128, kappa=2.0,
                                          kappa_length=0, alpha_1=100.0, alpha_2=20.0, sigma_1=0.02,
                                          scale_nominal=True, x_dim=10, cayley=True)
    backbone = make_ortho_KWLarge_Concat(out_dim=10, act="GroupSort")
    sampler = CompositeSampler((10,), [UniformSimplexSampling(), CorrectConeSampling()])
    sched = CompositeSamplerScheduler([LinearScheduler(-0.02, 1.0, "min", 0.02, 10),
                                       LinearScheduler(0.02, 0.0, "max", 0.98, 10)], [1.0, 1.0])
    mod = LyapunovLearning(order=1, h_sample_size=h_sample, h_dist_lim=15.0, sampler=sampler,
                           sampler_scheduler=sched, dynamics=dyn, init_fun=UniformInitFun((10,), backbone),
                           lya_cand=DecisionBoundary(on_simplex=True), t_max=1.0, opt_name="Adam", lr=5e-3,
                           train_ode=train_ode, train_ode_epoch=TRAIN_ODE_EPOCH,
                           train_ode_solver=solver if train_ode else "dopri5",
                           train_ode_tol=(0.1 if solver == "rk4" else 1e-3) if train_ode else 1e-3,
                           val_ode_solver="dopri5", val_ode_tol=1e-3,
                           weight_decay=0.0, warmup=-1, max_epochs=300, simplex=True, act="relu", val_adv=False,
                           seed=seed)
    mod.current_epoch = EPOCH
    mod.dyn_fun.scale_nominal = False      # switched off at epoch_off_scale=10 (pl_modules.py:392-393)
    return mod.to(dev).train()


def cpu_baseline(budget_s: float = 25.0, images: int = B_PER_RANK, train_ode: bool = True, max_steps: int = 20,
                 warmup: int = 3):
    """The SAME training step as the GPU number beside it, on the host cores: B=128 images at
    epoch 20 (204 uniform + 52 correct-cone rows per image), the KWLarge-Cayley backbone forward
    and backward (the restated module's NCHW torch path), the dynamics' Cayley maps, the reference
    fan-out restated op for op in torch (oracle/torch_ref.py: Exp(1) samplers, dropout masks,
    jvp(DecisionBoundary, eval_dot) through the QP autograd Function with dense (N,C,C) Jacobians,
    hinge, the no-grad logging pass), the train_ode RK4 solve (10 steps / 40 train-mode evals,
    autograd through the stages, loss mix), backward and Adam.  BASELINE.md section 5: median of
    the timed steps after ``warmup`` warm-ups; at most ``max_steps`` (20) timed steps, fewer when
    the ``budget_s`` bound is reached (the count is reported)."""
    threads = int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0))))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    cpu = torch.device("cpu")
    # the reference's cayley() inverts with torch.inverse; the product's inverse is the HIP kernel
    # (no CPU path), so this host-side timing leg swaps in torch.linalg.inv while it runs
    from fiode_amd import cayley as CY
    hip_inverse, CY._block_inverse = CY._block_inverse, torch.linalg.inv
    try:
        return _cpu_baseline_run(budget_s, images, train_ode, max_steps, warmup, cpu)
    finally:
        CY._block_inverse = hip_inverse


def _cpu_baseline_run(budget_s, images, train_ode, max_steps, warmup, cpu):
    import statistics
    from oracle import torch_ref as T
    threads = torch.get_num_threads()
    mod = build_module(cpu, seed=0, train_ode=train_ode)
    mod.parallel_cayley = False
    opt = torch.optim.Adam(mod.parameters(), lr=5e-3)
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(images, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (images,), generator=g)
    S, S1 = H_SAMPLE, 204
    S2 = S - S1
    p_ode = min(0.98, (EPOCH - TRAIN_ODE_EPOCH) / 50.0)
    h0 = torch.full((images, 10), 0.1)

    def one():
        opt.zero_grad(set_to_none=True)
        feat = mod.init_coordinates.param_map(x)                       # backbone
        W = mod.dyn_fun.effective_weights()                           # Cayley maps of the dynamics
        with torch.no_grad():                                          # CompositeSampler + nn.Dropout masks
            hu = T.uniform_simplex(torch.empty(S1, 10).exponential_(generator=g))
            hc = T.correct_cone(torch.empty(images, S2, 10).exponential_(generator=g), y)
            h = torch.cat([hu[None].expand(images, -1, -1), hc], 1).flatten(0, 1)
            N = images * S
            m = [torch.rand(N, 128, generator=g) >= 0.5 for _ in range(4)]
        loss, eff, ma = T.lyapunov_loss(h, feat, y, S, W, scale_nominal=False, kappa=2.0, p=0.5, mask1=m[0],
                                        mask2=m[1], lmask1=m[2], lmask2=m[3])
        if train_ode:
            with torch.no_grad():
                om = (torch.rand(40, 2, images, 128, generator=g) >= 0.5)
            loss_ode, _ = T.ode_train_loss(feat, h0, y, W, om, 0.0, 1.0, 0.1, scale_nominal=False, p=0.5)
            loss = loss * (1.0 - p_ode) + loss_ode * p_ode
        loss.backward()
        opt.step()

    for _ in range(warmup):
        one()
    times = []
    t_all = time.perf_counter()
    while len(times) < max_steps and (len(times) < 3 or time.perf_counter() - t_all < budget_s):
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    dt = statistics.median(times)
    what = ("the full configs[1] training step" if train_ode else "the full Lyapunov-only training step")
    return {"value": round(images / dt, 2), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"median of {len(times)} steps (after {warmup} warm-ups) of {what} at B={images} x "
                      f"S={H_SAMPLE} (S1=204/S2=52) on the host: backbone fwd/bwd + Cayley maps + the reference "
                      f"fan-out restated op for op in torch (oracle/torch_ref.py)" +
                      (" + train_ode RK4 (40 evals) with autograd through the stages" if train_ode else "") +
                      f" + Adam, float32, {dt * 1e3:.1f} ms/step (same workload as value)"}


def load_pmc(kernel: str) -> dict:
    """Counter-derived figures of `kernel` from the committed rocprofv3 --pmc summary
    (profiles/pmc_summary.json, written by tools/prof_summary.py from separate --pmc passes of this
    bench command): HBM bytes per launch and the MFMA-busy fraction.  They are NOT measured in this
    run (a --pmc pass perturbs the timing); "pmc_source" names the pass they come from."""
    p = ROOT / "profiles" / "pmc_summary.json"
    if not p.exists():
        return {}
    try:
        d = json.loads(p.read_text())
    except Exception:
        return {}
    k = d.get(kernel, {})
    return {"traffic": k.get("hbm_bytes_per_launch"), "mfma_busy": k.get("mfma_busy_frac"),
            "lds_bank_conflict_frac": k.get("lds_bank_conflict_frac"), "pmc_source": d.get("_source")}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """``--gpus N`` (N > 1) without a launcher around us: start N rank processes as CHILDREN
    (torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1) -- the reference's
    ``Trainer(gpus=N, accelerator='ddp')`` spawns its ranks the same way (sl_pipeline.py:157-170).
    Called before this process touches the GPU (no exec: the parent waits and relays).  Rank 0's
    JSON line is checked (n_gpus == N, parallelism dpN) and re-printed; anything else on the ranks'
    stdout goes to stderr.  Returns the exit code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py")] + argv
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, cwd=str(ROOT))
    lines = []
    for line in proc.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            lines.append(s)
        else:
            print(line, end="", file=sys.stderr, flush=True)
    rc = proc.wait()
    if rc != 0:
        print(f"bench.py: rank processes exited with {rc}", file=sys.stderr)
        return rc
    if len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    rec = json.loads(lines[0])
    if rec.get("n_gpus") != n or rec.get("config", {}).get("parallelism") != f"dp{n}":
        print(f"bench.py: refusing a line with n_gpus={rec.get('n_gpus')} for --gpus {n}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=25.0)
    ap.add_argument("--prof-reps", type=int, default=20)
    ap.add_argument("--eager", action="store_true", help="dispatch the step op by op (no hipGraph replay)")
    ap.add_argument("--workload", choices=("rk4", "lyap"), default="rk4",
                    help="rk4: BASELINE configs[1] (Lyapunov loss + differentiable RK4 train_ode solve); "
                         "lyap: the Lyapunov-only step")
    ap.add_argument("--no-secondary", action="store_true", help="skip the Lyapunov-only companion measurement")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the configs[3] (certification) and configs[4] (B=1024 x S=1024) companion lines")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: the line would misreport n_gpus")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # RCCL ("nccl") between GPUs; FIODE_BENCH_BACKEND=gloo rehearses the N-rank path with
        # several ranks sharing the visible GPUs (device = local rank mod device count)
        dist.init_process_group(backend=os.environ.get("FIODE_BENCH_BACKEND", "nccl"), init_method="env://")
    dev = torch.device(f"cuda:{local % max(1, torch.cuda.device_count())}")
    torch.cuda.set_device(dev)

    def timed_run(train_ode: bool, steps: int, warmup: int, solver: str = "rk4", batch: int = B_PER_RANK,
                  h_sample: int = H_SAMPLE, strict: bool = True):
        """Build the module, capture (or not) the step, run warmup + timed steps; max over ranks."""
        mod = build_module(dev, seed=0, train_ode=train_ode, solver=solver, h_sample=h_sample)
        mod.seed = 1000 + rank                      # each rank draws its own samples / dropout masks
        opt = mod.configure_optimizers(capturable=not args.eager)[0][0]
        params = [p for p in mod.parameters() if p.requires_grad]
        g = torch.Generator(device="cpu").manual_seed(1234 + rank)
        x = torch.rand(batch, 3, 32, 32, generator=g).to(dev)
        y = torch.randint(0, 10, (batch,), generator=g).to(dev)
        from fiode_amd.distributed import GradAllReducer, MetricReducer, broadcast_parameters
        broadcast_parameters(mod)                   # DDP's construction-time broadcast
        reducer = GradAllReducer(params) if world > 1 else None   # p.grad = views into one flat bucket
        metrics = MetricReducer(["training_loss", "effective_batch_size", "mean_active_constraints"], dev)

        def sync_metrics():
            sc = mod.last_plan["scalars"]
            metrics.reduce({"training_loss": sc[0], "effective_batch_size": sc[1],
                            "mean_active_constraints": sc[2]}, world)   # fused sync_dist

        last = {}
        if args.eager:
            def step():
                opt.zero_grad(set_to_none=False)
                loss = mod.compute_loss(x, y, batch, "relu")
                loss.backward()
                if world > 1:
                    reducer.allreduce(world)          # one RCCL all-reduce of the whole gradient
                    sync_metrics()
                opt.step()
                mod.global_step += 1
                last["loss"] = loss
        else:
            from fiode_amd.graph_step import GraphTrainStep
            # comm: RCCL collectives captured in the step ("graph", the default over nccl) or eager
            # between two replays ("eager"); FIODE_COMM overrides (e.g. a runtime that cannot capture)
            # placement_trials: the fastest of a few captures on different side streams (the executor's
            # hardware-queue placement of the step's branches; GraphTrainStep._select_placement)
            gstep = GraphTrainStep(mod, opt, x, y, reducer=reducer, world=world, comm=os.environ.get("FIODE_COMM"),
                                   placement_trials=int(os.environ.get("FIODE_PLACEMENT_TRIALS", "4")))
            last["placement_ms"] = gstep.placement_ms
            last["recaptures"] = getattr(gstep, "placement_recaptures", 0)
            last["comm"] = gstep.comm if world > 1 else None

            def step():
                last["loss"] = gstep.step()           # hipGraph replay (+ eager RCCL between graphs)
                if world > 1:
                    sync_metrics()

        for _ in range(warmup):
            step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        # health of the timed run, read after the timed region: the sticky status of the persistent
        # train_ode solve (a timed-out QP-exit exchange poisons the loss with NaN) and the last loss
        health = {"status": int(mod.device_status()) if hasattr(mod, "device_status") else 0,
                  "loss_finite": bool(torch.isfinite(last["loss"]).all()),
                  "skipped_steps": gstep.skipped_steps() if not args.eager else 0}
        # skipped_steps: replays whose update the step guard skipped (a non-finite loss -- e.g.
        # log(y_hat) of a dopri5 interpolant that undershoots 0, which the reference would feed to
        # Adam as NaN -- or a failed solve); reported, the timed work was done
        if strict and (health["status"] or not health["loss_finite"]):
            raise RuntimeError(f"unhealthy timed run: {health}")
        # a companion line (strict=False) whose steps were skipped or whose solve failed did not
        # train (a failed solve may even stop early): it is marked invalid, never a throughput claim
        why = [k for k, bad in (("solve status", health["status"] != 0), ("non-finite loss", not health["loss_finite"]),
                                ("guard-skipped steps", health["skipped_steps"] > 0)) if bad]
        health["valid"] = not why
        if why:
            health["invalid_reason"] = ", ".join(why)
        health["comm"] = last.get("comm")
        if last.get("placement_ms") is not None:
            health["placement_ms"] = last["placement_ms"]     # per trial capture; the fastest is kept
            health["placement_recaptures"] = last.get("recaptures", 0)
        return float(dt.item()), mod, x, y, health

    def certify_companion(n_img: int = 2):
        """BASELINE configs[3]: certify_lipschitz (certify_lipschitz.py:97-143) of this rank's images on
        the T=40 decision-boundary grid (G = 41,320,837 rows, resident in HBM, built once), 10
        batches + the 7-row tail, the QP exit per batch; images sharded over the ranks (each rank
        certifies n_img images, the count all-reduce is outside the timed region)."""
        from fiode_amd import ops
        from fiode_amd.certify import certify_lipschitz
        grid = ops.certify_grid(40, device=dev)
        G = int(grid.shape[0])
        cmod = build_module(dev, seed=0, train_ode=False)
        g = torch.Generator(device="cpu").manual_seed(4321 + rank)
        xs = torch.rand(n_img + 1, 3, 32, 32, generator=g).to(dev)
        ys = torch.randint(0, 10, (n_img + 1,), generator=g).to(dev)
        certify_lipschitz(cmod, xs, ys, T=40, grid=grid, indices=[0])        # warm-up image
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = certify_lipschitz(cmod, xs, ys, T=40, grid=grid, indices=range(1, n_img + 1))
        torch.cuda.synchronize()
        dtc = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.barrier()
            dist.all_reduce(dtc, op=dist.ReduceOp.MAX)
        ms = float(dtc.item()) / n_img * 1e3
        flop = FLOP_ROW_FWD_PASS * G                 # one MLP per grid row (the QP pass reuses it)
        tf = flop / (ms * 1e-3) / 1e12
        del grid
        torch.cuda.empty_cache()
        return {"ms_per_image": round(ms, 3), "images_per_s": round(world * n_img / (n_img * ms * 1e-3), 3),
                "grid_rows": G, "grid_rows_per_s": round(world * G / (ms * 1e-3), 1),
                "mlp_tflops": round(tf, 3), "frac": round(tf / MFMA_F32_PEAK_TFLOPS, 4), "images_per_rank": n_img,
                "max_violation": [round(v, 4) for v in res.max_violations],
                "workload": "BASELINE configs[3]: certify_lipschitz on the T=40 decision-boundary grid, one image "
                            "at a time (backbone + grid forward + QP per batch + violation max), images "
                            f"sharded over {world} rank(s); TFLOP/s = 37,888 FLOP x G over the whole per-image "
                            "time (all four kernels)"}

    train_ode = args.workload == "rk4"
    elapsed, mod, x, y, health = timed_run(train_ode, args.steps, args.warmup)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B_PER_RANK * args.steps / elapsed
    lyap_only = dopri5_step = None
    if train_ode and not args.no_secondary:
        e2, _, _, _, _ = timed_run(False, args.steps, args.warmup)
        lyap_only = {"images_per_s": round(world * B_PER_RANK * args.steps / e2, 2),
                     "ms_per_step": round(e2 / args.steps * 1e3, 4)}
        # BASELINE configs[2]: the same train step with the YAML's own train_ode solver (dopri5, tol
        # 1e-3: cifar_train.yaml:30,32), backprop through the adaptive solve
        e3, m3, _, _, h3 = timed_run(True, args.steps, args.warmup, solver="dopri5", strict=False)
        st3 = m3.last_ode_plan["stats"].cpu().tolist()
        dopri5_step = {"valid": h3["valid"], "images_per_s": round(world * B_PER_RANK * args.steps / e3, 2),
                       "ms_per_step": round(e3 / args.steps * 1e3, 4), "device_status": h3,
                       "last_solve": {"nfe": st3[0], "n_accept": st3[4], "n_reject": st3[5]},
                       "workload": "BASELINE configs[2]: the configs[1] step with train_ode_solver dopri5, "
                                   "train_ode_tol 1e-3 (rtol = atol), direct backprop through the adaptive solve"}
    certify_line = large_batch = None
    if not args.no_configs:
        certify_line = certify_companion()
        # BASELINE configs[4]: B=1024 images x h_sample 1024 per rank, train_ode dopri5 (tol 1e-3),
        # backbone + Cayley maps + Adam, DDP over the ranks (the same bucketed all-reduce)
        k4 = max(1, min(args.steps, 10))
        e4, m4, _, _, h4 = timed_run(True, k4, 2, solver="dopri5", batch=1024, h_sample=1024, strict=False)
        st4 = m4.last_ode_plan["stats"].cpu().tolist()
        large_batch = {"valid": h4["valid"], "images_per_s": round(world * 1024 * k4 / e4, 2),
                       "ms_per_step": round(e4 / k4 * 1e3, 4),
                       "steps": k4, "rows_per_rank": 1024 * 1024, "device_status": h4,
                       "last_solve": {"nfe": st4[0], "n_accept": st4[4], "n_reject": st4[5]},
                       "workload": "BASELINE configs[4]: train step at B=1024 x h_sample 1024 per rank (S1=819 "
                                   "uniform + 205 correct-cone rows/image), train_ode dopri5 tol 1e-3, "
                                   f"KWLarge-Cayley backbone + Adam, dp{world}"}
        del m4
        torch.cuda.empty_cache()

    # ---- per-kernel timing of the fused hot path with HIP events (same inputs as a step) ----
    from fiode_amd import _lib as L, ops
    with torch.no_grad():
        feat = mod.init_coordinates.param_map(x).float().contiguous()
        w = {k: v.detach().float().contiguous() for k, v in mod.dyn_fun.effective_weights().items()}
    plan = mod.step_plan(y)
    nk = len(L.LYAP_KERNELS)
    tot = [0.0] * nk
    for r in range(args.prof_reps + 2):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(nk + 1)]
        torch.cuda._sleep(4_000_000)
        ops.lyap_step(feat, y, w, plan["dyn"], sample_size=plan["S"], n_uniform=plan["S1"], sampler=plan["sampler"],
                      dropout_mode=plan["dropout_mode"], kappa=plan["kappa"], seed=plan["seed"], offset=r, events=evs)
        torch.cuda.synchronize()
        if r >= 2:
            for i in range(nk):
                tot[i] += evs[i].elapsed_time(evs[i + 1])
    kern_ms = {L.LYAP_KERNELS[i]: tot[i] / args.prof_reps for i in range(nk)}
    rows = B_PER_RANK * H_SAMPLE
    kern_flop = {k: FLOP_ROW[k] * rows for k in FLOP_ROW}
    if train_ode:
        # the differentiable RK4 solve: k_ot_fwd (one kernel) and k_ot_bwd + its wgrad chain
        oplan = mod.ode_plan(B_PER_RANK)
        h0 = torch.full((B_PER_RANK, 10), 0.1, device=dev)
        E = ops.odetrain_evals(oplan["cfg"])
        t_f = t_b = 0.0
        for r in range(args.prof_reps + 2):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            # keep the stream busy while the host enqueues, so e0..e2 time GPU work only (not the
            # host's allocation / argument packing between the event records)
            torch.cuda._sleep(4_000_000)
            e0.record()
            yo, _, ws = ops.odetrain_forward(feat, h0, w, oplan["dyn"], oplan["cfg"], offset_dev=oplan["offset_dev"])
            e1.record()
            ops.odetrain_backward(torch.ones_like(yo), feat, w, oplan["dyn"], oplan["cfg"], ws)
            e2.record()
            torch.cuda.synchronize()
            if r >= 2:
                t_f += e0.elapsed_time(e1)
                t_b += e1.elapsed_time(e2)
        # the forward launched at this batch: 4-row tiles (k_ot_fwd4) up to 1,024 rows (odetrain.hip)
        fwd_name = "k_ot_fwd4" if (B_PER_RANK + 3) // 4 <= 256 else "k_ot_fwd"
        kern_ms[fwd_name] = t_f / args.prof_reps
        kern_ms["k_ot_bwd+wgrad"] = t_b / args.prof_reps
        kern_flop[fwd_name] = FLOP_ROW_FWD_PASS * E * B_PER_RANK
        kern_flop["k_ot_bwd+wgrad"] = (2 * (10 * 128 + 128 * 128 + 128 * 10) + FLOP_ROW_FWD_PASS) * E * B_PER_RANK
    hot_ms = sum(kern_ms.values())
    dom = max(kern_flop, key=lambda k: kern_ms[k])
    ach = kern_flop[dom] / (kern_ms[dom] * 1e-3) / 1e12
    pmc = load_pmc(dom)
    roofline = {"bound": "mfma", "achieved": round(ach, 3), "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / MFMA_F32_PEAK_TFLOPS, 4), "traffic": pmc.get("traffic"),
                "mfma_busy": pmc.get("mfma_busy"), "lds_bank_conflict_frac": pmc.get("lds_bank_conflict_frac"),
                "pmc_source": pmc.get("pmc_source"), "kernel": dom,
                "kernel_ms": round(kern_ms[dom], 4), "flop_per_launch": kern_flop[dom],
                "per_kernel_ms": {k: round(v, 4) for k, v in kern_ms.items()},
                "per_kernel_tflops": {k: round(kern_flop[k] / (kern_ms[k] * 1e-3) / 1e12, 3)
                                      for k in kern_flop},
                "hot_path_tflops": round(sum(kern_flop.values()) / (hot_ms * 1e-3) / 1e12, 3)}
    out = {"metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32", "data": "synthetic (x~U[0,1) 128x3x32x32 per rank, y~randint(10))",
           "config": {"workload": ("hipGraph replay" if not args.eager else "eager") + ": " + (
                          "BASELINE configs[1]: train step of README.md:27 at epoch 20 with train_ode (rk4, step_size "
                          "0.1, t_max=1: 10 steps / 40 train-mode f-evals, backprop through the stages; loss_ode "
                          "portion 0.2) + the Lyapunov loss (B=128, h_sample_size=256 -> 204 uniform + 52 "
                          "correct-cone rows/image), KWLarge-Cayley backbone + Adam" if train_ode else
                          "Lyapunov-only train step of README.md:27 at epoch 20 (B=128, h_sample_size=256 -> 204 "
                          "uniform + 52 correct-cone rows/image), KWLarge-Cayley backbone + Adam"),
                      "global_batch": world * B_PER_RANK, "h_sample_size": H_SAMPLE,
                      "rows_per_rank": rows, "parallelism": f"dp{world}"},
           "roofline": roofline,
           "hot_path": {"ms": round(hot_ms, 4), "images_per_s": round(world * B_PER_RANK / (hot_ms * 1e-3), 1)},
           "lyapunov_only_step": lyap_only,
           "dopri5_train_step": dopri5_step,
           "certify_T40": certify_line,
           "large_batch_step": large_batch,
           "process_group": {"backend": dist.get_backend() if world > 1 else None, "world_size":
                             dist.get_world_size() if world > 1 else 1},
           "device_status": health,
           "runtime_env": {"DEBUG_HIP_FORCE_GRAPH_QUEUES": os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES")}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_budget, train_ode=train_ode)
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
