"""The training step as replayable hipGraphs (torch.cuda.CUDAGraph = hipGraph on ROCm).

One eager step of the README model launches ~1,000 kernels from Python (backbone FFT convs,
Cayley maps, autograd, Adam); at B=128 the GPU work is a few ms, so the eager step is bound by
host dispatch.  The whole step has no host synchronisation (the fused fan-out, the QP exit and
the Cayley inverses are all device-side), so it is captured once and replayed:

* ``fwd_bwd`` graph: zero grads -> compute_loss (backbone, Cayley maps, fused fan-out kernels)
  -> backward, accumulating into the persistent ``p.grad`` tensors (with a GradAllReducer these
  are views into its flat bucket) -> advance the device Philox counter, so every replay draws
  fresh samples and dropout masks;
* ``opt`` graph: the Adam step (``capturable=True``: step counts on the device);
* maps_ahead: the conv layers' Cayley maps of the NEXT step are computed inside this one (see
  ``_maps_ahead_on``).
For one rank both are captured into a single graph.  For N ranks over RCCL (comm "graph") too:
the gradient buffer is laid out in the order the warm-up backward finalised the gradients and
cut into ~4 MB buckets, and each bucket's all-reduce is captured on a comm stream as soon as its
last gradient is final (GradAllReducer.arm / finish), so the collectives of the early buckets (the
dynamics, the head and the 4096 -> 512 CayleyLinear) overlap the rest of the backward (the conv
stack) -- DDP's bucketed overlap (sl_pipeline.py:157-170), one replay per step.  Over gloo
(comm "eager": not capturable) the bucket all-reduces run between two replays.

Step guard: the optimizer kernel (FiodeAdam) skips the update on the device -- p, m, v and the
step counts untouched, one more in the sticky ``skipped`` word -- when this step's train_ode solve
failed (its status words: attempt capacity exhausted, an exchange timed out) or its loss is not
finite; on N ranks each rank's verdict rides in the all-reduced gradient bucket's guard slot, so
all ranks skip together.  ``check_status()`` (every ``check_every`` replays and on demand) raises
once a step was skipped.  (torch.amp's found_inf skip, without a host sync.)

Static inputs: ``step(x, y)`` copies the batch into the captured input buffers.  What the
captured step bakes in (and ``GraphTrainStep`` checks on every call): the sampler plan of the
current epoch (S1/S2 split, ``scale_nominal``), the kappa ramp's anchor (the ramp itself follows the
device step counter),
batch shape.  Recapture (construct a new GraphTrainStep) at an epoch boundary.
"""
from __future__ import annotations

from typing import Optional

import os

import torch

from .streams import distinct, new_stream

# priority of the stream the step is captured on (its nodes' hardware queue; tools/ab_step.py cap_hi)
CAPTURE_PRIORITY = 0
# zeroed GEMM workspace slots reserved per capture (streams made in it that run split-K GEMMs)
CAPTURE_WS_SLOTS = 24



# The HIP runtime of this image (ROCm 7.x, torch's libamdhip64) dereferences a null internal stream in
# its graph executor when a captured graph has more parallel branches than it can place on
# GPU_MAX_HW_QUEUES < 4 hardware queues: a host SIGSEGV at the first replay (tools/probes/
# hwq_branch_probe.py: any K-branch graph, K >= 2 at 1 queue, K >= 3 at 2, K = 6 / 12 at 3; none
# up to K = 12 at the default 4).  The training step's graph has more branches than that (map
# prefetch, the ODE solve, the conv maps computed ahead), so the capture is refused up front.
MIN_HW_QUEUES = 4


def _check_runtime_queues() -> None:
    import os
    q = os.environ.get("GPU_MAX_HW_QUEUES")
    if q is not None and q.strip().isdigit() and int(q) < MIN_HW_QUEUES:
        raise RuntimeError(f"GraphTrainStep: GPU_MAX_HW_QUEUES={q} < {MIN_HW_QUEUES}: this HIP runtime's graph "
                           "executor segfaults replaying a multi-branch graph with fewer hardware queues "
                           "(DESIGN.md section 6); unset it or use >= 4")


class GraphTrainStep:
    def __init__(self, module, optimizer, x: torch.Tensor, y: torch.Tensor, *, reducer=None, world: int = 1,
                 warmup: int = 3, act: str = "relu", check_every: int = 200, maps_ahead: bool = True,
                 comm: Optional[str] = None, bucket_bytes: int = 4 << 20, force_comm: bool = False,
                 guard: bool = True, placement_trials: int = 1, warm_capture: bool = True):
        _check_runtime_queues()
        dev = x.device
        if dev.type != "cuda":
            raise ValueError("GraphTrainStep needs ROCm device tensors")
        self.module, self.opt, self.reducer, self.world, self.act = module, optimizer, reducer, world, act
        self.check_every, self.n_replays = int(check_every), 0
        self.piped, self.early = [], False
        # N ranks: "graph" = the bucket all-reduces captured in the step (RCCL); "eager" = between
        # replays (gloo, or any backend on request).  force_comm: run the collectives even at
        # world 1 (the capture path's test on one GPU).
        self.force_comm = bool(force_comm)
        multi = reducer is not None and (world > 1 or self.force_comm)
        if comm is None:
            import torch.distributed as dist
            comm = "graph" if (multi and dist.is_initialized() and dist.get_backend() == "nccl") else "eager"
        if comm not in ("graph", "eager"):
            raise ValueError(f"comm must be 'graph' or 'eager', got {comm!r}")
        self.comm = comm if multi else "none"
        self.comm_stream = new_stream(dev) if self.comm == "graph" else None
        dyn = module.dyn_fun
        if module.rng_counter is None:
            module.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        # the kappa ramp (pl_modules.py:447-448) follows the device step counter in the captured
        # step: global_step = rng_counter + anchor (LyapunovLearning.kappa_device)
        ramp = dyn.kappa_length and module.global_step < dyn.kappa_length
        module._kappa_anchor = (module.global_step - int(module.rng_counter.item())) if ramp else None
        self.epoch = module.current_epoch
        self.static_x = x.detach().clone()
        self.static_y = y.detach().clone()
        if module.rng_counter is None:
            module.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.skipped = torch.zeros(1, dtype=torch.int32, device=dev)     # sticky count of guarded skips
        self._guard_ok = guard and hasattr(optimizer, "guard")          # FiodeAdam / FiodeAdamW
        # Grads are set to None before every backward, so autograd hands its result tensors over
        # (no zero fills, no per-parameter accumulate adds); inside the graph they come from the
        # graph's private pool at fixed addresses.  N ranks: one multi-tensor copy then moves them
        # into the reducer's flat bucket (GradAllReducer.gather) and p.grad points at the bucket
        # views, which the RCCL all-reduce and the optimizer graph use.
        self.persistent = False
        self.single = world == 1 and not self.force_comm

        # Warm-up iterations (lazy optimizer state, library handles, workspaces) run real updates on
        # the constructor's batch; the reference's Lightning loop makes no such updates, so the
        # parameters, the optimizer state and the Philox counter are restored afterwards (in place:
        # the captured graph must see the tensors the warm-up created).
        snap = self._snapshot()
        side = new_stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for it in range(warmup):
                if it == 0 and multi:
                    reducer.record_order()          # the order the backward finalises the gradients
                self._fwd_bwd(bucket_plan=False)
                if it == 0 and multi:
                    reducer.plan_buckets(reducer.recorded_order(), bucket_bytes)
                self._between()
                self.opt.step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self._restore(snap)
        self.skipped.zero_()
        torch.cuda.synchronize(dev)

        if maps_ahead:
            self._maps_ahead_on()
        # every capture (the first one included) on fresh dedicated streams made in the same order, so
        # the placement trials compare like with like.  warm_capture: the first capture in a process
        # replays ~10 % slower than any later capture of the same step (same kernels, same launch
        # shapes -- profiles/r06/warm_capture.json: placement trials 1.349 / 1.226 / 1.236 / 1.228 ms
        # without, 1.243 / 1.241 / 1.244 / 1.242 with one discarded capture ahead), so one capture is
        # made and dropped first (no kernel runs in a capture: parameters, optimizer state and
        # counters are untouched; every rank does the same, so captured collectives stay paired).
        self.comm_fallback = None
        for keep in ([False, True] if warm_capture else [True]):
            self._fresh_streams()
            try:
                self._capture()
            except Exception as exc:               # noqa: BLE001 - rethrown unless it is the comm capture
                if self.comm != "graph":
                    raise
                # the collectives could not be captured by this runtime: eager bucket all-reduces
                # between two graphs instead (the reason is kept in comm_fallback)
                if self.reducer is not None:
                    self.reducer._armed = None
                self.comm, self.comm_fallback = "eager", repr(exc)
                self._capture()
            if not keep:
                # The dropped capture's autograd graph stays referenced (self.loss), so the
                # parameters' AccumulateGrad nodes made in it -- bound to its capture stream -- serve
                # the kept captures too; that binding is what makes them replay faster: freeing the
                # graph first brings the slow first-capture time back (1.348 vs 1.239 ms,
                # profiles/r06/warm_capture.json).  torch warns about the stream mismatch it causes
                # (an extra event join per parameter inside the graph): silenced, it is deliberate.
                self.g_fb = self.g_opt = None
                torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        self.placement_ms = None
        if placement_trials > 1 and self.comm != "eager":
            self._select_placement(int(placement_trials))
        if self.reducer is not None and (world > 1 or self.force_comm):
            views = [self.reducer.flat.data_ptr() <= p.grad.data_ptr() < self.reducer.flat.data_ptr()
                     + self.reducer.flat.numel() * self.reducer.flat.element_size() for p in self.params]
            if not all(views):
                raise RuntimeError("p.grad does not point into the reducer's bucket after capture")
        self.scalars = module.last_plan["scalars"]
        # a float lr is a launch argument baked into the captured optimizer step (a tensor lr is
        # read on the device: LR schedulers may change it between replays)
        self._float_lrs = [g["lr"] for g in self.opt.param_groups]

    def _select_placement(self, trials: int, reps: int = 12) -> None:
        """Keep the fastest of ``trials`` captures of the same step on different side streams.

        The hipGraph executor runs each captured stream's nodes on that stream's hardware queue, and
        which of the 4 queues a stream has is fixed when the stream is made: with the step's branches
        (the Cayley maps' chains, the train_ode solve, the conv stack) landing on shared queues in
        different ways, one capture of the same graph replays in 1.51 ms and another in 1.94 ms, and
        a recapture on the same streams reproduces its time (tools/probes/placement_probe.py,
        DESIGN.md section 4).  Each trial captures on fresh pool streams for the module's map
        prefetch and ODE solve and times a few replays; the winner's streams are restored and
        captured again.  Every trial replays from the same state, and the replays' updates are undone
        (parameters, optimizer state, Philox counter, step count, maps computed ahead) -- the results
        of the kept graph are those of any capture, bit for bit."""
        import time
        m = self.module
        snap = self._snapshot()
        gstep = m.global_step

        def replay():
            self.g_fb.replay()
            if not self.one_graph:
                self._between(warmup=False)
                self.g_opt.replay()

        def clock():
            # every trial replays from the same state (the adaptive solve's NFE follows the state)
            self._restore(snap)
            m.global_step = gstep
            self.refresh_maps()
            best = float("inf")
            for _ in range(2):
                for _ in range(2):
                    replay()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(reps):
                    replay()
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t) / reps)
            return best

        stores = [c._store for c in self.piped if getattr(c, "_store", None) is not None]

        def streams():
            return (getattr(m, "_side_streams", None), getattr(m, "_ode_stream", None),
                    [st["stream"] for st in stores], getattr(self, "capture_stream", None))

        def use(sv):
            m._side_streams, m._ode_stream, conv, self.capture_stream = sv
            for st, cs in zip(stores, conv):
                st["stream"] = cs

        dev = self.static_x.device
        trials_t = [(clock(), streams())]
        for _ in range(trials - 1):
            # fresh pool streams for the maps' prefetch, the ODE solve, the conv maps computed ahead
            # and the capture itself
            self._fresh_streams()
            self._capture()
            trials_t.append((clock(), streams()))
        times = [t for t, _ in trials_t]
        import torch.distributed as dist
        if dist.is_initialized() and dist.get_world_size() > 1:
            # N ranks: one decision for all (the slowest rank's time per trial), so every rank
            # captures the same number of times -- the captured collectives stay in step
            tt = torch.tensor(times, dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            times = tt.tolist()
        best = min(range(len(times)), key=lambda i: times[i])
        self.placement_recaptures = 0
        if best != len(trials_t) - 1:
            use(trials_t[best][1])
            self._capture()
            # the recapture on the winner's streams replays like its trial -- but once a bench read
            # 1.322 ms after a 1.218 ms trial (profiles/r06/warm_capture.json): check it and capture
            # again (at most twice) when it is > 3 % off (N ranks: one decision, the slowest rank's)
            for _ in range(2):
                t = clock()
                if dist.is_initialized() and dist.get_world_size() > 1:
                    tt = torch.tensor([t], dtype=torch.float64, device=dev)
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                    t = float(tt.item())
                if t <= times[best] * 1.03:
                    break
                self._capture()
                self.placement_recaptures += 1
        torch.cuda.synchronize()
        self._restore(snap)
        m.global_step = gstep
        self.skipped.zero_()
        self.n_replays = 0
        self.refresh_maps()
        torch.cuda.synchronize()
        self.placement_ms = [round(t * 1e3, 4) for t in times]
        self.placement_pick = best

    def _fresh_streams(self) -> None:
        """New dedicated streams (fiode_amd.streams) for the module's map prefetch and ODE solve
        (made at their first use in the capture), the conv maps computed ahead and the capture."""
        m, dev = self.module, self.static_x.device
        m._side_streams = m._ode_stream = None
        for c in self.piped:
            if getattr(c, "_store", None) is not None:
                c._store["stream"] = new_stream(dev)
        self.capture_stream = new_stream(dev, priority=CAPTURE_PRIORITY)

    def role_streams(self) -> list:
        """Every stream a capture of this step forks work to: the capture stream, the module's map
        prefetch / ODE / weight-tap streams, the conv maps' streams, the comm stream and the
        module-level head stream."""
        from . import cayley as CY
        m = self.module
        out = [getattr(self, "capture_stream", None), getattr(self, "comm_stream", None),
               getattr(m, "_ode_stream", None), getattr(m, "_wtap_stream", None)]
        out += list(getattr(m, "_side_streams", None) or [])
        out += [c._store["stream"] for c in self.piped if getattr(c, "_store", None) is not None]
        out += list(CY._HEAD_STREAMS.values())
        return out

    def _capture(self):
        # two roles on one HIP stream can make a stream that joined the capture wait on an event it
        # recorded itself, which this ROCm runtime answers with a host SIGSEGV in hipStreamEndCapture
        # (streams.py); the product's streams are dedicated, so this only trips on a caller's own
        if not distinct(self.role_streams()):
            raise RuntimeError("GraphTrainStep: two roles of the captured step share one HIP stream "
                               "(use fiode_amd.streams.new_stream for side streams, not the torch pool)")
        self.one_graph = self.single or self.comm == "graph"
        # zeroed split-K counter words for the GEMMs of streams this capture makes (ops._Workspace:
        # taken from an arena zeroed here, not filled by the replay on the step's chain)
        from . import ops
        ops._Workspace.reserve(self.static_x.device, CAPTURE_WS_SLOTS)
        # capture_error_mode "thread_local": the process group's watchdog thread polls its events
        # during our capture; in the default "global" mode such a call from ANOTHER thread aborts it
        # ("operation not permitted when stream is capturing" -> the watchdog terminates the process)
        self.g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fb, stream=getattr(self, "capture_stream", None),
                              capture_error_mode="thread_local"):
            self.loss = self._fwd_bwd()
            if self.one_graph:
                self.opt.step()
                self._refresh_late()
        self.g_opt = None
        if not self.one_graph:
            self.g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_opt, stream=getattr(self, "capture_stream", None),
                                  capture_error_mode="thread_local"):
                self.opt.step()
                self._refresh_late()

    # ---- conv maps computed ahead -------------------------------------------------------------
    # Each CayleyConv's spectral map depends only on its own two parameters, and the step's first
    # convolution waits for it.  With maps_ahead the map of step t+1 is computed at the end of step
    # t into fixed buffers (CayleyConv.pipeline_on): on one rank inside the backward, as soon as the
    # layer's gradient is final (its map backward), the layer's parameters get their Adam update
    # (FiodeAdam.step_params) and the next map is computed on the layer's stream while the rest of
    # the backward runs; on N ranks (gradients final only after the all-reduce) after the optimizer
    # step.  The maps are the same kernels on the same parameters as at the start of the next step,
    # so the results are unchanged.  Parameters changed outside the replays: call refresh_maps().
    # The early per-layer update needs the layer's map backward to run ONCE per step with the
    # layer's whole gradient: with the reference-order second backbone pass
    # (ode_reuse_features False) each layer has two map nodes per step, so there the maps are
    # refreshed after the optimizer step instead (late refresh, correct for any number of uses).
    def _maps_ahead_on(self):
        from .cayley import CayleyConv
        from .optim import _KernelStepMixin, _kernel_ok_params
        once = getattr(self.module, "ode_reuse_features", True) or not getattr(self.module, "train_ode", False)
        self.early = self.single and once and isinstance(self.opt, _KernelStepMixin)
        root = getattr(self.module, "init_coordinates", self.module)       # the backbone's layers
        for c in root.modules():
            if isinstance(c, CayleyConv) and c.pipeline_on():
                self.piped.append(c)
        if self.early and not all(_kernel_ok_params(self.opt, [c.weight, c.alpha]) for c in self.piped):
            self.early = False          # a group the kernel does not cover: update in step()
        if self.early:
            for c in self.piped:
                c._store["on_grads"] = (lambda gw, ga, c=c: self._update_layer(c, gw, ga))

    def _update_layer(self, c, gw, ga):
        self.opt.step_params([(c.weight, gw), (c.alpha, ga)])
        c.refresh_map()

    def _refresh_late(self):
        if not self.early:
            for c in self.piped:
                c.refresh_map()

    def refresh_maps(self) -> None:
        """Recompute the maps computed ahead from the current parameters (after loading a
        checkpoint or any update outside the replays)."""
        for c in self.piped:
            c.refresh_map()

    def close(self) -> None:
        """Back to maps computed at the start of each step (eager training of the same module), and
        the optimizer's step guard disarmed: the guard reads this graph's loss / status / slot
        tensors, which no later eager step writes, so a guard left armed would keep skipping (or
        keep passing) on a stale verdict."""
        self.module._kappa_anchor = None
        for c in self.piped:
            c.pipeline_off()
        self.piped = []
        self._disarm_guard()

    def _disarm_guard(self) -> None:
        if hasattr(self.opt, "guard"):
            self.opt.guard = None
        if self.reducer is not None and hasattr(self.reducer, "guard_writer"):
            self.reducer.guard_writer = None

    def _snapshot(self):
        """Copies of what a warm-up iteration changes: parameters, optimizer state (None where a
        parameter has none yet), the device Philox counter."""
        with torch.no_grad():
            params = [p.detach().clone() for p in self.params]
            state = []
            for p in self.params:
                st = self.opt.state.get(p)
                state.append(None if not st else {k: (v.detach().clone() if torch.is_tensor(v) else v)
                                                  for k, v in st.items()})
            counter = self.module.rng_counter.detach().clone()
        return params, state, counter

    def _restore(self, snap):
        params, state, counter = snap
        with torch.no_grad():
            for p, v in zip(self.params, params):
                p.copy_(v)
            for p, old in zip(self.params, state):
                st = self.opt.state.get(p)
                if not st:
                    continue
                for k, v in st.items():
                    if not torch.is_tensor(v):
                        if old is not None and k in old:
                            st[k] = old[k]
                        continue
                    if old is not None and k in old and torch.is_tensor(old[k]):
                        v.copy_(old[k])
                    else:
                        v.zero_()        # state created by the warm-up: its initial value (Adam: 0)
            self.module.rng_counter.copy_(counter)

    def _fwd_bwd(self, bucket_plan: bool = True):
        m = self.module
        for p in self.params:
            p.grad = None
        overlap = self.comm == "graph" and bucket_plan
        if overlap:
            self.reducer.arm(self.world, self.comm_stream, force=self.force_comm)
        loss = m.compute_loss(self.static_x, self.static_y, self.static_x.shape[0], self.act)
        self._arm_guard(loss)
        loss.backward(self._unit_grad(loss))
        if overlap:
            self.reducer.finish()                 # the last buckets, join the comm stream, 1/world
        elif self.comm != "none":
            self.reducer.gather()                 # one multi-tensor copy into the flat bucket
        m.rng_counter.add_(1)
        return loss

    def _unit_grad(self, loss):
        """The backward seed d loss / d loss = 1 as a fixed tensor made outside the capture and marked
        (lyapunov.UNIT_GRAD), so the captured step has no fill kernel for it and the fused loss node
        skips its scaling by it."""
        from .lyapunov import UNIT_GRAD
        u = getattr(self, "_unit", None)
        if u is None or u.device != loss.device or u.dtype != loss.dtype:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("GraphTrainStep: the unit gradient seed must exist before the capture")
            u = torch.ones((), dtype=loss.dtype, device=loss.device)
            setattr(u, UNIT_GRAD, True)
            self._unit = u
        return u

    def _arm_guard(self, loss):
        """Point the optimizer's step guard at this step's loss and solve status words (they are new
        tensors in every eager iteration; fixed graph-pool tensors inside the capture)."""
        if not self._guard_ok:
            self._disarm_guard()            # no guard of an earlier GraphTrainStep on this optimizer
            return
        from .optim import StepGuard
        status = self.module.status_words() if hasattr(self.module, "status_words") else []
        lo = loss.detach().reshape(1)
        mine = StepGuard(loss=lo if lo.dtype == torch.float32 else None, status=status)
        if self.comm != "none":
            # N ranks: this rank's verdict goes into the bucket's guard slot (written right before
            # the last bucket's all-reduce); the optimizer reads the summed slot
            self.reducer.guard_writer = mine.write_flag
            self.opt.guard = StepGuard(flag=self.reducer.guard_slot, skipped=self.skipped)
        else:
            mine.skipped = self.skipped
            self.opt.guard = mine

    def _between(self, warmup: bool = True):
        # eager collectives: every warm-up iteration (the captured step has none of its own when
        # comm is "graph"), and between the two replays when comm is "eager"
        if self.comm == "eager" or (self.comm == "graph" and warmup):
            self.reducer.allreduce(self.world, force=self.force_comm)

    def step(self, x: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None):
        m = self.module
        if m.current_epoch != self.epoch:
            raise RuntimeError("epoch changed: the captured sampler plan is stale, recapture the step")
        for g, lr in zip(self.opt.param_groups, self._float_lrs):
            if not torch.is_tensor(lr) and g["lr"] != lr:
                raise RuntimeError(f"learning rate changed since capture ({lr} -> {g['lr']}): the captured step "
                                   "bakes a float lr in; use a tensor lr (Adam(..., lr=torch.tensor(lr, "
                                   "device=...), capturable=True)) or recapture the step")
        if x is not None:
            self.static_x.copy_(x, non_blocking=True)
        if y is not None:
            self.static_y.copy_(y, non_blocking=True)
        self.g_fb.replay()
        if not self.one_graph:
            self._between(warmup=False)
            self.g_opt.replay()
        m.global_step += 1
        self.n_replays += 1
        if self.check_every > 0 and self.n_replays % self.check_every == 0:
            self.check_status()
        return self.loss

    def skipped_steps(self) -> int:
        """Replayed steps whose optimizer update the guard skipped (one host read)."""
        return int(self.skipped.item())

    def check_status(self) -> None:
        """Raise if a replayed step was skipped by the guard (a failed train_ode solve or a
        non-finite loss, on any rank) or the last solve reports a failure (one or two host reads,
        every ``check_every`` replays and on demand)."""
        n = self.skipped_steps()
        if n:
            st = self.module.device_status() if hasattr(self.module, "device_status") else 0
            raise RuntimeError(f"{n} training step(s) skipped by the step guard (failed train_ode solve or "
                               f"non-finite loss; last solve status {st}): parameters and optimizer state "
                               "are those of the last good step")
        if hasattr(self.module, "check_device_status"):
            self.module.check_device_status()
