"""Distributed runner: one process per GPU (or per CPU rank), torchrun-style env.

GPU ranks: torch.distributed only bootstraps.  By default every rank exports
an IPC descriptor of its fine-grained xGMI mailbox, the descriptors are
all-gathered once, and afterwards each step's exchange (halo columns to the
strip neighbours + every rank's dt, MIN-folded on device) runs on the device:
fused into the inviscid and lean N-S tile kernels (edge cells push, the last
workgroup's wavefront publishes and waits), or as hf2d_p2p_push / unpack
after the mechanism step (DeviceSolver p2p transport).  ``transport="rccl"``
(or HF2D_TRANSPORT=rccl) instead issues pack + grouped ncclSend/ncclRecv +
unpack on the solver stream.  Either way the inner loop never returns to
Python and is captured in step graphs.

CPU ranks (tests, gloo): the native CpuSolver calls back into Python for the
halo columns and the scalar reductions, which go over torch.distributed.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from ..models.simulation import maybe_autotune, parse_fault
from .strips import balanced_columns


def init_from_env(backend: Optional[str] = None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* env vars."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group(backend=backend or "gloo", rank=rank, world_size=world)
    return rank, world


def any_rank(flag, device: bool = False) -> bool:
    """True on every rank if ``flag`` is true on any rank (all-reduce MAX).

    For host loops whose trip count must agree across ranks although their
    condition is rank-local -- bench.py's step-graph priming: each rank's
    autotune picks graphs on or off from its own timings, and every step
    exchanges with the other ranks, so a rank-local loop condition deadlocked a
    4-rank run (profiles/bench_rehearsal_shared_gpu_r06.txt).  ``device``: the
    process group is NCCL/RCCL (the flag travels as a device tensor)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32)
    if device:
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item()) == 1


class DistributedSimulation:
    """A strip of a deck run on this rank."""

    def __init__(self, deck_text: str, backend: str = "gpu", *, rank: int = 0, world: int = 1,
                 device: int = 0, semantics: str = "mpi", fused: bool = True, lean: bool = True, parts=None,
                 workdir: str = ".", use_checkpoint: bool = False, transport: Optional[str] = None):
        from .. import native

        hf = native()
        self.hf = hf
        self.rank, self.world = rank, world
        if world > 1:
            self.case, self.parts = self._window_case(deck_text, workdir, use_checkpoint, semantics, parts)
        else:
            self.case = hf.Case.from_deck(deck_text, workdir, use_checkpoint)
            self.case.set_semantics(semantics)
            self.parts = parts or balanced_columns(np.asarray(self.case.field("solid")), world)
        gi0, gi1 = self.parts[rank]
        self.backend = backend
        self.transport = "none"
        self.p2p_validated = False
        self.p2p_error = ""
        if backend == "gpu":
            self.solver = hf.DeviceSolver(self.case, device, gi0, gi1)
            self.solver.fused = fused
            self.solver.lean = lean
            self.autotune_log = maybe_autotune(self.case, self.solver)
            if world > 1:
                self._wire_gpu(transport or os.environ.get("HF2D_TRANSPORT", "p2p"))
        elif backend == "cpu":
            self.solver = hf.CpuSolver(self.case, gi0, gi1)
            self.solver.lean = lean
            if world > 1:
                self._wire_cpu()
        else:
            raise ValueError(backend)
        if world > 1:
            # the backend holds the strip now: keep only it and one ghost column
            # each side on the host (outputs are written per strip, stripio.cpp)
            self.case.trim_to_columns(gi0 - 1, gi1 + 1)

    def _window_case(self, deck_text, workdir, use_checkpoint, semantics, parts):
        """Strip-local pre-processing: no rank ever holds the whole field
        (SURVEY 5.7).  Every rank runs the pre-processor's geometry over the
        whole grid on a 16 B/cell flag plane and builds the 1248 B records of
        its own columns (+ one ghost column each side) only
        (Case.from_deck_window); a restart reads the rank's slab of the .hf2d.
        The reference instead pre-processes on rank 0 and sends each rank its
        subdomain (hf2d_start.cpp:115-116,143-205).  The strips come from a
        flags-only pass (Case.partition_deck), identical on every rank, and
        the whole-field eligibility facts from every strip's part, gathered
        in rank order over a host (gloo) group."""
        import torch.distributed as dist

        rank, world = self.rank, self.world
        if not parts:
            parts = self.hf.Case.partition_deck(deck_text, workdir, use_checkpoint, world)
        parts = [tuple(p) for p in parts]
        a, b = parts[rank]
        nx = parts[-1][1]
        case = self.hf.Case.from_deck_window(deck_text, workdir, use_checkpoint, max(a - 1, 0), min(b + 1, nx))
        case.set_semantics(semantics)
        grp = None if dist.get_backend() == "gloo" else dist.new_group(backend="gloo")
        facts = [None] * world
        dist.all_gather_object(facts, case.facts_part(), group=grp)
        case.merge_facts(facts)
        if grp is not None:
            dist.destroy_process_group(grp)
        return case, parts

    # -- GPU transports -------------------------------------------------------
    def _wire_gpu(self, transport: str):
        """Per-step halo + dt exchange between the strip GPUs.

        ``p2p`` (default): xGMI peer-to-peer mailboxes -- the descriptors of
        every rank's IPC-exported mailbox are all-gathered here once, then each
        step exchanges with one device kernel (no RCCL launch, no host).
        ``rccl``: pack kernel + grouped ncclSend/ncclRecv + unpack kernel.
        Host-side reductions (output steps only) use RCCL when the process
        group is NCCL/RCCL, else torch.distributed callbacks.  If any rank
        cannot map its peers' mailboxes, every rank falls back to RCCL.
        """
        import torch
        import torch.distributed as dist

        if transport not in ("p2p", "rccl"):
            raise ValueError("transport must be p2p or rccl, got %r" % transport)
        s = self.solver
        rank, world = self.rank, self.world
        nccl = dist.get_backend() == "nccl"
        if nccl or transport == "rccl":
            obj = [self.hf.DeviceSolver.nccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            s.init_comm(obj[0], rank, world)
        else:
            s.set_comm(rank, world, *self._py_comm_funcs())
        self.transport = "rccl"
        if transport != "p2p":
            return
        ok = 1
        err = ""
        try:
            desc = s.p2p_export(rank, world)
        except Exception as e:  # pragma: no cover - hardware dependent
            desc, ok, err = b"", 0, str(e)
        descs = [None] * world
        dist.all_gather_object(descs, desc)
        if ok and all(descs):
            try:
                s.p2p_import(descs)
            except Exception as e:  # pragma: no cover - hardware dependent
                ok, err = 0, str(e)
        else:
            ok = 0
        if self._all_ok(ok, nccl):
            # self-validation: one exchange of the full state with poisoned
            # ghost columns and a rank-tagged dt, checksummed on every rank
            blobs = [None] * world
            dist.all_gather_object(blobs, s.p2p_probe())
            ok, why = self.hf.DeviceSolver.p2p_probe_ok(blobs, rank)
            if not ok:
                err = "self-validation failed: " + why
        if self._all_ok(ok, nccl):
            self.transport = "p2p"
            self.p2p_validated = True
            # the exchange is folded into the tile kernels (the last workgroup
            # publishes and waits, one peer per lane); HF2D_P2P_FUSE=0 selects a
            # separate exchange kernel.  Device-side cost per step without a
            # second strip on the GPU: tools/exchange_loopback.py
            # (profiles/exchange_loopback_r05.md)
            s.p2p_fuse = os.environ.get("HF2D_P2P_FUSE", "1") == "1"
        else:
            if not nccl:
                obj = [self.hf.DeviceSolver.nccl_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                s.init_comm(obj[0], rank, world)
            s.p2p_fallback()
            self.p2p_error = err
            if err:
                print("[hf2d rank %d] p2p transport unavailable (%s); using RCCL" % (rank, err), flush=True)

    @staticmethod
    def _all_ok(ok: int, nccl: bool) -> bool:
        import torch
        import torch.distributed as dist

        flag = torch.tensor([int(bool(ok))], dtype=torch.int32)
        if nccl:
            flag = flag.cuda()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return int(flag.item()) == 1

    def _py_comm_funcs(self):
        import torch
        import torch.distributed as dist

        rank, world = self.rank, self.world

        def fmin(v):
            t = torch.tensor([v], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return float(t.item())

        def fsum(v):
            t = torch.tensor([v], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            return float(t.item())

        def fmaxi(v):
            t = torch.tensor([v], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return int(t.item())

        def fres(b):
            arr = torch.frombuffer(bytearray(b), dtype=torch.uint8)
            out = [torch.empty_like(arr) for _ in range(world)]
            dist.all_gather(out, arr)
            return b"".join(bytes(o.numpy().tobytes()) for o in out)

        def fallgather(b):
            out = [None] * world
            dist.all_gather_object(out, bytes(b))
            return out

        return fmin, fsum, fmaxi, fres, fallgather

    # -- gloo wiring for the CPU stepper ------------------------------------
    def _wire_cpu(self):
        import torch
        import torch.distributed as dist

        s = self.solver
        rank, world = self.rank, self.world
        left, right = rank - 1, rank + 1

        def exchange(solver, group):
            n_loc = solver.local_nx
            first = solver.l_off
            last = solver.l_off + (solver.gi1 - solver.gi0) - 1
            ops = []
            bufs = {}
            if left >= 0:
                snd = torch.from_numpy(np.ascontiguousarray(solver.pack_column(group, first)))
                rcv = torch.empty_like(snd)
                ops += [dist.P2POp(dist.isend, snd, left), dist.P2POp(dist.irecv, rcv, left)]
                bufs["l"] = rcv
            if right < world:
                snd = torch.from_numpy(np.ascontiguousarray(solver.pack_column(group, last)))
                rcv = torch.empty_like(snd)
                ops += [dist.P2POp(dist.isend, snd, right), dist.P2POp(dist.irecv, rcv, right)]
                bufs["r"] = rcv
            if ops:
                for r in dist.batch_isend_irecv(ops):
                    r.wait()
            if "l" in bufs:
                solver.unpack_column(group, 0, bufs["l"].numpy())
            if "r" in bufs:
                solver.unpack_column(group, n_loc - 1, bufs["r"].numpy())

        s.set_exchange(exchange)
        s.set_comm(rank, world, *self._py_comm_funcs())

    def step(self, n: int, residual: bool = False):
        self.solver.run_steps(int(n), bool(residual))

    def run(self, max_cycles: int = 1, outdir: str = ".", outputs: bool = True, checkpoint: bool = True,
            verbose: bool = True, metrics: str = "", profile: str = "", fault: str = ""):
        """Full DEEPS driver (outer cycles, outputs on rank 0 after a strip gather)."""
        step, rank, kind = parse_fault(fault)
        return self.solver.run(max_cycles, outdir, outputs, checkpoint, verbose, metrics, profile, step, rank, kind)

    def summary(self):
        return dict(self.solver.summary())

    def gather_field(self, name: str) -> np.ndarray:
        """Full (nx, ny) field on every rank (for tests/outputs)."""
        self.solver.download()
        f = np.asarray(self.case.field(name))
        if self.world == 1:
            return f
        import torch
        import torch.distributed as dist

        gi0, gi1 = self.parts[self.rank]
        mine = np.zeros_like(f)
        mine[gi0:gi1] = f[gi0:gi1]
        t = torch.from_numpy(mine)
        if self.backend == "gpu" and dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t)
        return t.cpu().numpy()
