"""SPMD data parallelism over RCCL (our own communicator, ``parallel/comm.py``) / Gloo on CPU.

Reference: the only multi-GPU mechanism is ``torch.nn.DataParallel`` over 4 GPUs
(Runner_P128_QuantumNAT_onchipQNN.py:135-153, Test.py:70-97): single process, one
Python thread per GPU, the module re-replicated on EVERY forward (the 32 MiB FC
weight broadcast 9x per step), gradients reduced to GPU0 9x per step (one per
``backward()``), outputs gathered to GPU0.

MI355X design:
  * one process per GPU (torchrun-compatible env: RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_ADDR / MASTER_PORT); weights stay resident -- a single rank-0 broadcast at
    init replaces the per-call replicate;
  * each rank owns a contiguous shard of the HBM-resident dataset and samples it
    independently (weak scaling: per-GPU work fixed);
  * gradients live in flat buffers; each bucket is ONE all-reduce launched
    asynchronously the moment backward finalises it (FC bucket first, while the conv
    backward still runs), the averaging factor 1/world is fused into the optimizer;
  * xGMI is point-to-point (7 links/GPU): RCCL rings are per-link bound, so we send
    few, large messages -- the 33.6 MB FC gradient as a single bucket, all small
    parameter grads coalesced into one second bucket;
  * metrics (NMSE numerators/denominators, correct/total counts, loss sums) are
    all-reduced as raw sums -- the global NMSE is sum(err)/sum(pow), never a mean of
    per-rank ratios;
  * backends: "rccl" on GPUs -- one RCCL communicator per process (``parallel/comm.py``),
    every collective a stream-ordered RCCL kernel on a dedicated comm stream, with no
    process group, watchdog thread or work objects (so a HIP graph can capture the
    collectives with nothing polling them: docs/CONCURRENCY.md "captured collectives");
    "gloo" for CPU runs and the several-ranks-per-GPU rehearsal (torch.distributed);
    "torch_nccl" (QDML_DIST_BACKEND=torch_nccl) keeps torch's own ProcessGroupNCCL selectable as a
    fallback (eager / 5-graph plans only: its watchdog polls events, which a graph capture forbids);
  * failure detection (rccl): ``parallel/watchdog.py`` -- a thread with no HIP calls watches the
    heartbeat every completed host sync point bumps and RCCL's async-error state, and on a stall
    longer than QDML_PG_TIMEOUT or an error aborts the communicator and exits non-zero.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


_GLOO_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"   # none | rccl | gloo
    forced: bool = False   # collectives even at world 1 (QDML_FORCE_DIST=1: rehearses them)
    comm: Optional[object] = None    # (rccl) parallel.comm.RcclComm
    store: Optional[object] = None   # (rccl) the c10d store the communicator id travelled through
    watchdog: Optional[object] = None   # (rccl) parallel.watchdog.CommWatchdog
    _comm_stream: Optional[object] = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1 or self.forced

    @property
    def comm_stream(self) -> "torch.cuda.Stream":
        """(rccl) the one stream every gradient collective runs on: RCCL needs one issue order per
        communicator, and a single stream gives every rank the same one."""
        if self._comm_stream is None:
            self._comm_stream = torch.cuda.Stream(self.device)
        return self._comm_stream

    def _device_op(self, t: torch.Tensor, fn) -> torch.Tensor:
        """(rccl) run ``fn`` on a device tensor (host tensors round-trip through the device)."""
        if t.is_cuda:
            return fn(t)
        d = t.to(self.device)
        fn(d)
        t.copy_(d.cpu())
        return t

    def heartbeat(self, phase: Optional[str] = None) -> None:
        """A host sync point completed (the failure detector's heartbeat; ``phase``: what runs next)."""
        if self.watchdog is not None:
            self.watchdog.heartbeat(phase)

    def barrier(self) -> None:
        if not self.distributed:
            return
        if self.backend == "rccl":
            # a one-element all-reduce can only complete once every rank has issued it
            x = torch.ones(1, device=self.device)
            self.comm.all_reduce_(x)
            torch.cuda.current_stream(self.device).synchronize()
        elif self.backend == "torch_nccl":
            dist.barrier(device_ids=[self.device.index])
        else:
            dist.barrier()
        self.heartbeat()

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.distributed:
            if self.backend == "rccl":
                return self._device_op(t, lambda d: self.comm.broadcast_(d, src))
            dist.broadcast(t, src)
        return t

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.distributed:
            if self.backend == "rccl":
                self._device_op(t, lambda d: self.comm.all_reduce_(d, op))
                if not t.is_cuda:   # (a host result: the collective has completed)
                    self.heartbeat()
                return t
            dist.all_reduce(t, op=_GLOO_OPS[op])
        return t

    def max_scalar(self, v: float) -> float:
        return self.max_vector([v])[0]

    def max_vector(self, vs: Sequence[float]) -> List[float]:
        """Element-wise max over ranks of a short host vector (one collective)."""
        if not self.distributed:
            return [float(v) for v in vs]
        t = torch.tensor(list(vs), dtype=torch.float64)
        self.all_reduce_(t, "max")
        return [float(x) for x in t.tolist()]


_CTX: Optional[DistContext] = None


def check_local_gpus(local_rank: int, local_world: int, n_gpus: int) -> None:
    """RCCL needs one GPU per rank OF THIS NODE: the ranks of a node (LOCAL_WORLD_SIZE, torchrun's
    per-node count) must fit its visible GPUs.  The global WORLD_SIZE is irrelevant -- a 2 x 8 job has
    WORLD_SIZE 16 on 8-GPU nodes."""
    if local_rank >= n_gpus or local_world > n_gpus:
        raise RuntimeError(f"RCCL needs one GPU per rank: LOCAL_RANK={local_rank}, LOCAL_WORLD_SIZE={local_world} "
                           f"but {n_gpus} visible GPU(s) on this node (QDML_DIST_BACKEND=gloo rehearses several "
                           "ranks per GPU)")


def resolve_timeout(timeout_s: Optional[float] = None) -> float:
    """The rendezvous bound and the failure detector's stall timeout: ``timeout_s``, else ``QDML_PG_TIMEOUT``."""
    if timeout_s is not None:
        return float(timeout_s)
    from .watchdog import default_timeout_s
    return default_timeout_s()


def init_distributed(device: str = "auto", timeout_s: Optional[float] = None) -> DistContext:
    """Initialise from torchrun-style env vars; world 1 needs no process group.  ``timeout_s`` bounds the
    rendezvous and is the failure detector's stall timeout; default ``QDML_PG_TIMEOUT`` (600 s)."""
    global _CTX
    if _CTX is not None:
        return _CTX
    timeout_s = resolve_timeout(timeout_s)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    use_cuda = (device in ("auto", "cuda")) and torch.cuda.is_available()
    if use_cuda:
        # (QDML_DIST_BACKEND=gloo rehearses several ranks on fewer GPUs: ranks share devices)
        local_dev = local % torch.cuda.device_count()
        torch.cuda.set_device(local_dev)
        dev = torch.device("cuda", local_dev)
    else:
        dev = torch.device("cpu")
    backend = "none"
    forced = world == 1 and os.environ.get("QDML_FORCE_DIST") == "1"
    comm = store = None
    if world > 1 or forced:
        backend = os.environ.get("QDML_DIST_BACKEND") or ("rccl" if use_cuda else "gloo")
        backend = {"nccl": "rccl"}.get(backend, backend)   # (torch's name for it on ROCm)
        if backend not in ("rccl", "gloo", "torch_nccl"):
            raise ValueError(f"QDML_DIST_BACKEND={backend!r}: rccl, gloo or torch_nccl")
        if backend in ("rccl", "torch_nccl"):
            if not use_cuda:
                raise RuntimeError(f"the {backend} backend needs a GPU")
            check_local_gpus(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)), torch.cuda.device_count())
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if forced and "MASTER_PORT" not in os.environ:
            import socket
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        tmo = datetime.timedelta(seconds=timeout_s)
        if backend == "rccl":
            from .comm import RcclComm
            # (the env:// rendezvous: torchrun's agent store when there is one, else rank 0 hosts a TCPStore)
            store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world, timeout=tmo))
            comm = RcclComm(rank, world, dev, store)
        elif backend == "torch_nccl":
            # (the fallback: torch's ProcessGroupNCCL = RCCL on ROCm, with torch's own watchdog)
            dist.init_process_group("nccl", rank=rank, world_size=world, timeout=tmo, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world, timeout=tmo)
    wd = None
    if comm is not None and os.environ.get("QDML_WATCHDOG", "1") != "0":
        from .watchdog import CommWatchdog
        wd = CommWatchdog(comm, rank, timeout_s, poll_s=float(os.environ.get("QDML_WATCHDOG_POLL", "2"))).start()
    _CTX = DistContext(rank, world, local, dev, backend, forced, comm, store, wd)
    if comm is not None:
        _CTX.barrier()   # (every rank holds the communicator id: rank 0's store may go)
    return _CTX


def get_context() -> DistContext:
    return _CTX if _CTX is not None else DistContext()


def shutdown() -> None:
    global _CTX
    if _CTX is not None:
        if _CTX.comm is not None:
            torch.cuda.synchronize(_CTX.device)
            if _CTX.watchdog is not None:   # (before the communicator goes: it must not abort a closed one)
                _CTX.watchdog.stop()
            _CTX.comm.close()
        elif dist.is_initialized():
            dist.destroy_process_group()
    _CTX = None




class _Issued:
    """(rccl) a launched collective: the event recorded after it, the stream it ran on, and a process-wide
    sequence number (the identity GradBuckets' wait dedupe keys on: an id() of a freed event can be reused)."""
    __slots__ = ("event", "stream", "seq")
    _next = 0

    def __init__(self, event, stream):
        self.event, self.stream = event, stream
        self.seq = _Issued._next
        _Issued._next += 1


class GradBuckets:
    """Asynchronous all-reduce of named gradient buckets.

    A bucket is a list of flat fp32 tensors; a single tensor is reduced in place, several
    are coalesced through a staging buffer (one collective either way).  ``launch(name)``
    enqueues the collective after everything already on the current stream (RCCL's stream
    waits on it); ``wait()`` makes the current stream wait for all launched collectives and
    scatters coalesced results back -- no host synchronisation anywhere.
    """

    # members up to which a coalesced bucket is scattered back one copy launch per member.  0: always the
    # single multi-tensor launch -- measured no slower in the step (it is off the critical path:
    # world-1 RCCL one-graph 0.4677/0.4722 vs 0.4705/0.4709 ms, 5-graph 0.5673/0.5678 vs 0.5726/0.5727,
    # profiles/r2_24_bucket_ab.txt)
    FOREACH_MIN = 0

    def __init__(self, ctx: DistContext, buckets: Dict[str, Sequence[torch.Tensor]]):
        self.ctx = ctx
        self.buckets = {k: list(v) for k, v in buckets.items()}
        self.staging: Dict[str, torch.Tensor] = {}
        for k, ts in self.buckets.items():
            if len(ts) > 1:
                self.staging[k] = torch.empty(sum(t.numel() for t in ts), device=ts[0].device, dtype=ts[0].dtype)
        self.pending: Dict[str, list] = {}
        # (rccl) the last collective issued: RCCL needs the collectives of one communicator in one order on every
        # rank and never two of them running at once, so each next collective -- on the comm stream or inline on
        # the caller's stream -- is ordered after it.  Reset once nothing is pending.
        self._last: Optional[_Issued] = None
        # (rccl) (stream handle, collective sequence number) pairs already waited for: under HIP graph capture a
        # stream must not take the same node as a dependency twice (a duplicate edge crashed hipStreamEndCapture,
        # r4_12; docs/CONCURRENCY.md "duplicate dependency edges")
        self._waited = set()

    def clear(self) -> None:
        """Forget every launched collective (each has been waited for by the stream that consumes it)."""
        self.pending.clear()
        self._last = None
        self._waited.clear()

    def assert_quiescent(self) -> None:
        """Raise if a launched collective has not been waited for (a graph capture must not begin with one
        in flight: its completion would be observed from inside the capture).  With nothing pending, the
        ordering event of the last collective is dropped too (a capture must not wait on an event recorded
        before it began)."""
        if self.pending:
            raise RuntimeError(f"gradient collectives still pending: {sorted(self.pending)}")
        self._last = None
        self._waited.clear()

    def _wait_on(self, s, rec: "_Issued") -> None:
        """Make stream ``s`` wait for ``rec`` unless it already does: recorded on ``s`` itself (stream order) or
        waited for before (no duplicate dependency edges under capture)."""
        key = (s.cuda_stream, rec.seq)
        if rec.stream.cuda_stream == s.cuda_stream or key in self._waited:
            return
        s.wait_event(rec.event)
        self._waited.add(key)

    def bucket_bytes(self) -> Dict[str, int]:
        return {k: sum(t.numel() * t.element_size() for t in ts) for k, ts in self.buckets.items()}

    def _collective(self, fn, inline: bool = False):
        """Issue one collective.  gloo: ``fn(None)`` is a torch.distributed async call returning its work.
        rccl: ``fn(stream)`` issues the RCCL kernel on the context's comm stream, forked from the current
        stream (so it sees every gradient written so far); the returned handle is an event on the comm
        stream that ``wait`` joins back -- under graph capture the fork and the join are graph edges.
        ``inline``: the kernel runs on the CURRENT stream instead (for a collective its stream waits for right
        away: no fork / join hop), after the previous collective."""
        if self.ctx.backend != "rccl":
            return fn(None)
        cur = torch.cuda.current_stream(self.ctx.device)
        if inline:
            s = cur
        else:
            s = self.ctx.comm_stream
            s.wait_stream(cur)
        last = self._last
        # ordered after the previous collective; nothing to add when it ran on s or on cur (which s just joined)
        if last is not None and last.stream.cuda_stream not in (s.cuda_stream, cur.cuda_stream):
            self._wait_on(s, last)
        fn(s)
        ev = torch.cuda.Event()
        ev.record(s)
        self._last = _Issued(ev, s)
        return self._last

    def _all_reduce(self, t: torch.Tensor, inline: bool = False):
        if self.ctx.backend == "rccl":
            return self._collective(lambda s: self.ctx.comm.all_reduce_(t, stream=s), inline)
        return dist.all_reduce(t, async_op=True)

    def launch(self, name: str, inline: bool = False) -> None:
        """All-reduce bucket ``name``.  ``inline`` (rccl): on the current stream, which waits for it next."""
        if not self.ctx.distributed or name not in self.buckets:
            return
        ts = self.buckets[name]
        if len(ts) == 1:
            self.pending[name] = [self._all_reduce(ts[0], inline), None, None]
        else:
            st = self.staging[name]
            torch.cat([t.reshape(-1) for t in ts], out=st)
            self.pending[name] = [self._all_reduce(st, inline), st, ts]

    def launch_all(self) -> None:
        for k in self.buckets:
            self.launch(k)

    # -- sharded (ZeRO-1 style) collectives: one flat region split into `world` equal shards ----
    def _shard_staging(self, key: str, full: torch.Tensor) -> torch.Tensor:
        w = self.ctx.world
        if full.numel() % w:
            raise ValueError(f"sharded region of {full.numel()} elements not divisible by world {w}")
        st = self.staging.get(key)
        if st is None or st.numel() * w != full.numel() or st.dtype != full.dtype:
            st = self.staging[key] = torch.empty(full.numel() // w, device=full.device, dtype=full.dtype)
        return st

    def launch_reduce_scatter(self, name: str, full: torch.Tensor) -> None:
        """Sum ``full`` over ranks keeping only this rank's shard ``full.view(world, -1)[rank]`` (the
        other shards are left as they were).  The collective writes a shard-sized staging buffer that
        ``wait`` copies back into the shard (out of place: no reliance on in-place aliasing rules)."""
        if not self.ctx.distributed:
            return
        st = self._shard_staging("rs:" + name, full)
        if self.ctx.backend == "rccl":
            work = self._collective(lambda s: self.ctx.comm.reduce_scatter(st, full, stream=s))
        else:
            work = dist.reduce_scatter_tensor(st, full, async_op=True)
        self.pending[name] = [work, st, [full.view(self.ctx.world, -1)[self.ctx.rank]]]

    def launch_all_gather(self, name: str, full: torch.Tensor) -> None:
        """Every rank's shard of ``full`` to every rank (the inverse of the reduce-scatter layout).
        This rank's shard is staged first, so the collective never reads the buffer it writes."""
        if not self.ctx.distributed:
            return
        st = self._shard_staging("ag:" + name, full)
        st.copy_(full.view(self.ctx.world, -1)[self.ctx.rank])
        if self.ctx.backend == "rccl":
            work = self._collective(lambda s: self.ctx.comm.all_gather(full, st, stream=s))
        else:
            work = dist.all_gather_into_tensor(full, st, async_op=True)
        self.pending[name] = [work, None, None]

    def wait(self, names: Optional[Sequence[str]] = None) -> None:
        """Make the CURRENT stream wait for the named (default: all) launched collectives; a coalesced
        bucket is scattered back (once) on the first stream that waits for it, and a later waiter on another
        stream waits for that scatter-back (an event) -- not only for the collective.  A bucket may be waited
        for from several streams."""
        for k in list(self.pending) if names is None else [n for n in names if n in self.pending]:
            ent = self.pending[k]
            if isinstance(ent[0], _Issued):   # (rccl: join the collective's stream)
                self._wait_on(torch.cuda.current_stream(self.ctx.device), ent[0])
            else:
                ent[0].wait()
            if ent[1] is not None:
                # every member back from the staging buffer.  Few members: one copy launch each -- the
                # multi-tensor launch gives each 64K-element chunk ONE workgroup, so the conv gradient
                # member (~60K floats) was a single-workgroup copy of 40 us on the step's critical path
                # (profiles/r2_23_dp_one_graph_world1_kernel_stats.md); many members: one launch
                sizes = [t.numel() for t in ent[2]]
                parts = list(ent[1][:sum(sizes)].split(sizes))
                if len(sizes) <= self.FOREACH_MIN:
                    for t, src in zip(ent[2], parts):
                        t.view(-1).copy_(src)
                else:
                    torch._foreach_copy_([t.view(-1) for t in ent[2]], parts)
                ent[1] = None
                if ent[2][0].is_cuda:   # later waiters on OTHER streams must wait for the scatter-back too
                    ev = torch.cuda.Event()
                    ev.record()
                    ent.append(ev)
            elif len(ent) > 3:
                torch.cuda.current_stream().wait_event(ent[3])
        if names is None:
            self.clear()


class DeviceSampler:
    """Per-rank shuffled mini-batch indices over an HBM-resident shard (reference:
    DataLoader(shuffle=True) over the zipped 9-stream dataset, R:88-93).  Partial last
    batches are kept, as with drop_last=False."""

    def __init__(self, n: int, batch: int, device, seed: int = 0, rank: int = 0, shuffle: bool = True,
                 drop_last: bool = False):
        self.n, self.batch, self.device = n, batch, device
        self.seed, self.rank, self.shuffle, self.drop_last = seed, rank, shuffle, drop_last
        self.epoch = 0

    def __len__(self) -> int:
        return self.n // self.batch if self.drop_last else (self.n + self.batch - 1) // self.batch

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator(device="cpu")
            g.manual_seed(self.seed * 1000003 + self.epoch * 7919 + self.rank)
            perm = torch.randperm(self.n, generator=g).to(self.device)
        else:
            perm = torch.arange(self.n, device=self.device)
        for i in range(len(self)):
            yield perm[i * self.batch:(i + 1) * self.batch]
