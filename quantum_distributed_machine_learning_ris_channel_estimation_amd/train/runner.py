"""``Y2HRunner``: the training orchestrator (reference: Runner_P128_QuantumNAT_onchipQNN.py).

Public surface kept from the reference:
  attributes  Pilot_num, data_len, SNRdb, num_workers, batch_size, batch_size_DML, lr,
              lr_decay, lr_threshold, n_epochs, print_freq, optimizer, train_test_ratio,
              train_QSC_losses, val_QSC_losses, val_QSC_accuracies          (R:20-38)
  methods     get_optimizer (R:40-46), get_data (R:48-73), get_dataloader_DML (R:75-95),
              get_HDCE_loss / get_HDCE_estimate (R:97-132),
              train_Conv_Linear_of_HDCE (R:134-283), get_SE_loss / get_SE_estimate
              (R:285-302), train_QSC_P128 (R:307-426)
  new         train_SC_P128 (the classical-SC trainer Test.py expects but the reference
              lacks), train_all, resume, DP over RCCL, HIP-graph captured steps.

The training methods run the fused engines of train/engine.py on HBM-resident data;
the host-side helpers (get_data, get_dataloader_DML, get_*_loss) remain for API
compatibility and tests.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F
import torch.optim as optim
from torch.utils.data import DataLoader

from ..config import RunnerConfig
from ..data.channel import pack_channel, pack_pilots
from ..data.datasets import (DatasetFolder_DML, DMLStore, load_or_generate_stream, make_dml_stores, split_stream)
from ..models.estimators import NMSELoss, QSC_P128, SC_P128
from ..ops.gather import StepGather
from ..ops.optim import FlatParamSpace, make_optimizer
from ..parallel.dp import DeviceSampler, GradBuckets, init_distributed
from ..parallel.watchdog import disarmed
from ..utils.metrics import MetricsLogger, to_db
from ..utils.profiling import GraphedStep
from . import checkpoint as ck
from .engine import ClassifierStep, HDCEModel, HDCEStep


class Y2HRunner:
    def __init__(self, cfg: Optional[RunnerConfig] = None, **overrides):
        cfg = cfg or RunnerConfig()
        if overrides:
            cfg.update_from_dict(overrides)
        self.cfg = cfg
        for k, v in cfg.to_dict().items():
            setattr(self, k, v)
        self.train_QSC_losses: List[float] = []
        self.val_QSC_losses: List[float] = []
        self.val_QSC_accuracies: List[float] = []
        self.train_SC_losses: List[float] = []
        self.train_HDCE_losses: List[float] = []
        self.val_HDCE_nmse: List[float] = []
        self._stores: Optional[Tuple[DMLStore, DMLStore]] = None
        self.ctx = None

    # ------------------------------------------------------------------ config sync
    def _sync_cfg(self) -> RunnerConfig:
        """Attribute writes (runner.lr = ...) win over the dataclass, as in the reference."""
        for k in self.cfg.to_dict():
            setattr(self.cfg, k, getattr(self, k))
        return self.cfg

    def _context(self):
        if self.ctx is None:
            self.ctx = init_distributed(self.device)
            # same seed on every rank: identical init (rank 0 broadcasts anyway); data order differs per rank
            torch.manual_seed(self.seed)
            np.random.seed(self.seed % (2 ** 32))
            if self.deterministic:
                torch.use_deterministic_algorithms(True, warn_only=True)
        return self.ctx

    def _log(self) -> MetricsLogger:
        ctx = self._context()
        return MetricsLogger(self.log_jsonl, ctx.rank, ctx.world)

    def _print(self, *a, **kw) -> None:
        if self._context().is_main:
            print(*a, **kw, flush=True)

    # ------------------------------------------------------------------ reference helpers
    def get_optimizer(self, parameters, lr):
        if self.optimizer == "adam":
            return optim.Adam(parameters, lr=lr)
        elif self.optimizer == "sgd":
            return optim.SGD(parameters, lr=lr, momentum=0.9)
        raise NotImplementedError("Optimizer {} not understood.".format(self.optimizer))

    def get_data(self, data_len, indicator, uid):
        st = load_or_generate_stream(self.data_dir, indicator, uid, self.Pilot_num, self.SNRdb, data_len,
                                     self.synthetic, self.seed)
        print("data loaded for scenario" + str(indicator) + " user" + str(uid) + "!")
        tr, va = split_stream([a.numpy() for a in st], self.train_test_ratio)
        return tr, va

    def get_dataloader_DML(self, data_len):
        tds, vds = [], []
        for s in range(self.n_scenarios):
            for u in range(self.n_users):
                td, vd = self.get_data(data_len, s, u)
                tds.append(td)
                vds.append(vd)
        train_loader = DataLoader(DatasetFolder_DML(*tds), batch_size=self.batch_size_DML, shuffle=True,
                                  num_workers=self.num_workers, pin_memory=torch.cuda.is_available())
        val_loader = DataLoader(DatasetFolder_DML(*vds), batch_size=self.batch_size_DML, shuffle=True,
                                num_workers=self.num_workers, pin_memory=torch.cuda.is_available())
        return train_loader, val_loader

    def _pack_td(self, td, device):
        Yp = td[0] if torch.is_tensor(td[0]) else torch.as_tensor(td[0])
        HL = td[1] if torch.is_tensor(td[1]) else torch.as_tensor(td[1])
        HP = td[2] if torch.is_tensor(td[2]) else torch.as_tensor(td[2])
        return (pack_pilots(Yp, self.Pilot_num).to(device), pack_channel(HL).to(device), pack_channel(HP).to(device))

    def get_HDCE_loss(self, td, Conv, CE, criterion, device):
        Yp_input, label_out, perfect_out = self._pack_td(td, device)
        Hhat = CE(Conv(Yp_input))
        return criterion(Hhat, label_out), criterion(Hhat, perfect_out)

    def get_HDCE_estimate(self, vd, Conv, CE, device):
        Yp_input, label_out, perfect_out = self._pack_td(vd, device)
        return CE(Conv(Yp_input)), label_out, perfect_out

    def get_SE_loss(self, td, CNN, device):
        pred, label = self.get_SE_estimate(td, CNN, device)
        return F.nll_loss(pred, label)

    def get_SE_estimate(self, td, CNN, device):
        Yp = td[0] if torch.is_tensor(td[0]) else torch.as_tensor(td[0])
        label_out = torch.as_tensor(td[3]).long().to(device).reshape(-1)
        return CNN(pack_pilots(Yp, self.Pilot_num).to(device)), label_out

    # ------------------------------------------------------------------ device data
    def device_stores(self) -> Tuple[DMLStore, DMLStore]:
        """HBM-resident train/val stores (this rank's shard)."""
        if self._stores is None:
            ctx = self._context()
            with disarmed("data generation"):   # (host-only, may outlast the stall timeout on a big data_len)
                tr, va = make_dml_stores(self.data_len, self.Pilot_num, self.SNRdb, self.train_test_ratio, ctx.device,
                                         self.data_dir, self.synthetic, self.seed, self.n_scenarios, self.n_users)
            if ctx.world > 1:
                if not self._dp_reference():   # (reference semantics: every rank slices the same global batches)
                    tr = tr.shard(ctx.rank, ctx.world)
                va = va.shard(ctx.rank, ctx.world, drop_remainder=False)   # (metrics are global sums)
            self._stores = (tr, va)
            self._print(f"Data Loaded! ({tr.n_streams} streams x {tr.n} train / {va.n} val samples per rank, "
                        f"device={ctx.device})")
        return self._stores

    def _dp_reference(self) -> bool:
        """DataParallel semantics (dp_semantics="reference"): each step is ONE global batch of batch_size_DML
        per stream, drawn from the same permutation on every rank and cut into world contiguous parts
        (torch.nn.DataParallel's scatter, R:144-148); the loss is that global batch's."""
        if self.dp_semantics not in ("weak", "reference"):
            raise ValueError(f"dp_semantics {self.dp_semantics!r}")
        return self.dp_semantics == "reference" and self._context().world > 1

    def _local_part(self, idx: torch.Tensor) -> torch.Tensor:
        """(reference semantics) this rank's contiguous part of a global batch of indices."""
        ctx = self._context()
        return idx.tensor_split(ctx.world)[ctx.rank] if self._dp_reference() else idx

    def _graphs_on(self) -> bool:
        """HIP-graph captured training steps: world 1, or N > 1 over RCCL with ``dp_graphs`` on (the bucketed
        all-reduces are launched from and waited for on the capturing stream, so they become graph nodes --
        the flagship one-graph DP plan's pattern).  ``auto`` means on only when the entry point's capture
        pre-flight passed on every rank (it sets QDML_DP_GRAPHS=1 before anything touched the GPU)."""
        ctx = self._context()
        if not (self.hip_graphs and ctx.device.type == "cuda"):
            return False
        if ctx.world == 1:
            return True
        if self.dp_graphs not in ("on", "off", "auto"):
            raise ValueError(f"dp_graphs {self.dp_graphs!r}")
        on = self.dp_graphs == "on" or (self.dp_graphs == "auto" and os.environ.get("QDML_DP_GRAPHS") == "1")
        return on and ctx.backend == "rccl"

    # ------------------------------------------------------------------ HDCE
    def _sync_bn_buffers(self, model: HDCEModel) -> None:
        """Every rank takes rank 0's BN running statistics and batch counters before evaluation and
        checkpointing: DataParallel keeps replica 0's buffers (data_parallel.py:88-90), so the
        evaluated / saved model is one model, not a per-rank mix.  (Training normalises with batch statistics:
        the running buffers never feed back into a step.)"""
        ctx = self._context()
        if ctx.distributed:
            for t in model.run_mean + model.run_var + [model._nbt]:
                ctx.broadcast_(t)

    def build_hdce(self) -> HDCEModel:
        ctx = self._context()
        model = HDCEModel(self.Pilot_num, ctx.device, self.dtype, self.n_scenarios)
        ctx.broadcast_(model.space.flat)
        return model

    @torch.no_grad()
    def eval_hdce(self, model: HDCEModel, store: DMLStore, batch: int = 1024) -> Tuple[float, float]:
        """Global val NMSE vs label and vs perfect (R:216-235): sum err / sum pow over ALL streams.  On the
        GPU (hdce_engine "hip") through the HIP inference engine (train/infer.py: conv / BN / ReLU kernels,
        the routed FC GEMM); elsewhere through the model's torch forward."""
        E, U = self.n_scenarios, self.n_users
        acc = torch.zeros(4, device=store.Yp.device, dtype=torch.float64)
        if store.Yp.is_cuda and self.hdce_engine == "hip" and store.n > 0:
            from .infer import HIPInference
            eng = getattr(self, "_val_engine", None)
            if eng is None or eng.model.E != model.E:
                eng = self._val_engine = HIPInference(model.convs, model.fc, self.Pilot_num, store.Yp.device,
                                                      chunk=min(2304, 144 * ((store.n + 143) // 144)))
            else:
                eng.refresh(model.convs, model.fc)
            for s in range(store.n_streams):
                expert = torch.full((store.n,), int(store.scen[s]), device=store.Yp.device, dtype=torch.int64)
                Y = eng.estimate(store.Yp[s], expert)
                lab, per = store.Hlabel[s], store.Hperf[s]
                acc += torch.stack([((Y - lab) ** 2).sum(), (lab ** 2).sum(), ((Y - per) ** 2).sum(),
                                    (per ** 2).sum()]).double()
            self._context().all_reduce_(acc)
            return float(acc[0] / acc[1]), float(acc[2] / acc[3])
        model.eval()
        for s in range(0, store.n, batch):
            idx = torch.arange(s, min(s + batch, store.n), device=store.Yp.device)
            Yp, HL, HP = store.gather(idx)
            b = idx.numel()
            A = model.features(Yp.view(E, U, b, *Yp.shape[2:]), training=False)
            Y = model.fc_forward(A).float()
            lab = HDCEModel.rows_from_streams(HL.view(E, U, b, -1))
            per = HDCEModel.rows_from_streams(HP.view(E, U, b, -1))
            acc += torch.stack([((Y - lab) ** 2).sum(), (lab ** 2).sum(), ((Y - per) ** 2).sum(),
                                (per ** 2).sum()]).double()
        self._context().all_reduce_(acc)
        model.train()
        return float(acc[0] / acc[1]), float(acc[2] / acc[3])

    def train_Conv_Linear_of_HDCE(self):
        cfg = self._sync_cfg()
        ctx = self._context()
        tr, va = self.device_stores()
        model = self.build_hdce()
        opt = make_optimizer(model.space, self.optimizer, self.lr)
        E, U, B = self.n_scenarios, self.n_users, self.batch_size_DML
        sp = model.space
        n_conv = sp.offsets[sp.names.index("CE.FC.weight")]
        # N > 1: the update split at the conv / FC boundary (the flagship DP plan's split): the FC part steps as
        # soon as its all-reduce -- launched before the conv backward, hidden behind it -- has landed, beside
        # the conv bucket's all-reduce; elementwise, so the split changes no value
        split = ctx.distributed
        if split:
            opt.partition([n_conv])
        model.attach_fc_shadow(opt)
        if self.hdce_engine not in ("hip", "torch"):
            raise ValueError(f"hdce_engine {self.hdce_engine!r}")
        hip = None if self.hdce_engine == "hip" else False
        ref = self._dp_reference()
        Bl = (B + ctx.world - 1) // ctx.world if ref else B   # (the first ranks' part of a global batch)
        step = HDCEStep(model, U, Bl, hip=hip)
        skip = step.skip if self.nan_guard else None
        # reference semantics: the global batch's per-stream NMSE denominators (every rank computes them from
        # the global indices); the ranks' losses are shares of ONE loss, so the gradients are SUMMED
        den_global = torch.zeros(E * U, 2, device=ctx.device) if ref else None
        rowpow = None
        # per-row label powers (GPU): the one-pass loss kernels and the FC GEMM's loss epilogue read them (the
        # hand-written FC paths -- incl. the fp8 estimator's e4m3 GEMMs -- need them)
        if ctx.device.type == "cuda" and step.hip:
            rowpow = (step.nmse._row_powers(tr.Hlabel), step.nmse._row_powers(tr.Hperf))
        # the NaN-guard flag rides in the conv bucket: all ranks skip (or step) together
        # the NaN-guard flag (final once the loss pass ends) travels in its own bucket right before the FC one,
        # so every rank skips -- or steps -- together, and the FC update need not wait for the conv bucket
        bk = {"fc": [sp.grad[n_conv:]], "conv": [sp.grad[:n_conv]]}
        if skip is not None:
            bk["skip"] = [skip]
        buckets = GradBuckets(ctx, bk)

        def grad_hook(name: str) -> None:
            if name == "fc":
                buckets.launch("skip")
            buckets.launch(name)
        step.grad_hook = grad_hook
        loss_acc = torch.zeros(2, device=ctx.device)
        last_loss = torch.zeros(2, device=ctx.device)
        static_idx = torch.zeros(B, dtype=torch.long, device=ctx.device)
        gscale = 1.0 if ref else 1.0 / ctx.world

        def part(n: int) -> int:
            """rows of a global batch of n this rank takes (torch.tensor_split's sizes in reference semantics)"""
            return n // ctx.world + (1 if ctx.rank < n % ctx.world else 0) if ref else n

        # one step engine + gather per part size, ALL built here, before any capture (an HDCEStep's constructor
        # synchronises the host): the full batch's part and the partial last batch's (drop_last=False)
        steps, gathers = {}, {}
        for n in sorted({B, tr.n % B or B}):
            b = part(n)
            if b > 0 and b not in steps:
                steps[b] = step if b == Bl else HDCEStep(model, U, b, grad_hook=grad_hook, skip=skip, hip=hip)
                gathers[b] = StepGather(E, U, b, model.H, model.W, ctx.device, with_classifier=False)

        def forward(idx):
            """gather + forward + loss of this rank's part of ``idx``; returns (step engine, loss) or None
            when the part is empty"""
            if ref:
                den_global[:, 0] = tr.Hlabel.index_select(1, idx).pow(2).sum((1, 2))
                den_global[:, 1] = tr.Hperf.index_select(1, idx).pow(2).sum((1, 2))
                idx = self._local_part(idx)
            b = idx.numel()
            if b == 0:
                return None
            g, hs = gathers[b], steps[b]
            g(tr, idx)
            hs.nmse.den_global = den_global
            if rowpow is not None:   # (the one-pass NMSE reads per-row label powers, scaled to global sums)
                g.rowpow = rowpow
                o = g.rowoff.long()
                g.rowden[:, 0] = rowpow[0][o]
                g.rowden[:, 1] = rowpow[1][o]
            return hs, hs.forward_fc_gathered(g, tr)

        def run(idx):
            sp.zero_grad()
            out = forward(idx)
            if out is None:
                # a partial last batch smaller than the world: this rank holds no rows, but still takes part
                # in every collective (zero gradients, a clear NaN flag) and in the optimizer step
                if skip is not None:
                    skip.zero_()
                grad_hook("fc")      # (the same collective order as every other rank)
                grad_hook("conv")
            else:
                hs, loss = out
                if hs.grad_hook:
                    hs.grad_hook("fc")
                hs.backward_conv()
                if hs.grad_hook:
                    hs.grad_hook("conv")
                last_loss.copy_(loss)
                loss_acc.add_(loss)
            if split:
                buckets.wait(("skip", "fc"))
                opt.step(grad_scale=gscale, skip=skip, part=1)
                buckets.wait(("conv",))
                opt.step(grad_scale=gscale, skip=skip, part=0)
                buckets.clear()
            else:
                buckets.wait()
                opt.step(grad_scale=gscale, skip=skip)

        def state():   # every tensor a step mutates
            return ([sp.flat, opt.m, opt.v, opt.step_t] + model.run_mean + model.run_var + [model._nbt, loss_acc]
                    + ([model.fc_shadow] if model.fc_shadow is not None else [])
                    + ([model.fp8_scales.amax, model.fp8_scales.scale, model.fp8_scales.qs]
                       if model.fp8_scales is not None else []))

        # fp8 estimator: seed the loss gradient's e4m3 scale from a bf16-gradient pass on a first batch
        # (forward returns the engine of this rank's part, or None for an empty part: that rank contributes amax 0
        # and still enters the max all-reduce, so no rank waits alone)
        step.prime_fp8_dy(lambda: (forward(torch.arange(min(B, tr.n), device=ctx.device)) or (None,))[0], state(), ctx,
                          engines=list(steps.values()))

        graphed = GraphedStep(lambda: run(static_idx), enabled=self._graphs_on())
        # (reference semantics: one permutation for every rank -- each takes its part of each global batch)
        sampler = DeviceSampler(tr.n, B, ctx.device, self.seed, 0 if ref else ctx.rank)
        d = ck.ckpt_dir(self.workspace, self.Pilot_num) if ctx.is_main else None
        log = self._log()
        best_nmse = 1000.0
        resume_path = os.path.join(ck.ckpt_dir(self.workspace, self.Pilot_num), f"HDCE_{B}_{self.SNRdb}dB_resume.pth")
        start = 0
        # (swa_epochs) the running sum of the per-epoch weight snapshots and their count
        swa = [torch.zeros_like(sp.flat), 0] if self.swa_epochs > 0 else None
        if self.resume:
            st = ck.load_resume(resume_path)
            if st is not None:
                ck.load_into(sp.flat, st["flat"])
                if swa is not None and "swa" in st:
                    ck.load_into(swa[0], st["swa"])
                    swa[1] = int(st["swa_n"])
                opt.load_state_dict(st["optimizer"])
                for t, v in zip(model.run_mean + model.run_var, st["run_mean"] + st["run_var"]):
                    ck.load_into(t, v)
                for t, v in zip(model.nbt, st["nbt"]):
                    ck.load_into(t, v)
                best_nmse, start = float(st["best"]), int(st["epoch"]) + 1
                self.train_HDCE_losses[:] = st["train_losses"].tolist()
                self.val_HDCE_nmse[:] = st["val_nmse"].tolist()
                if ctx.world == 1:
                    ck.set_rng_state(st["rng"])
                self._print(f"Resumed HDCE from {resume_path} at epoch {start}")
        self._print("Everything prepared well, start to train HDCE Conv+Linear...")
        for epoch in range(start, self.n_epochs):
            self._print(f"HDCE Conv+Linear:SNR: {self.SNRdb} Epoch [{epoch}]/[{self.n_epochs}] learning rate: "
                        f"{opt.lr:.4e}", time.strftime("%Y-%m-%d %H:%M:%S", time.localtime()))
            model.train()
            sampler.set_epoch(epoch)
            loss_acc.zero_()
            t0 = time.perf_counter()
            nb = 0
            for it, idx in enumerate(sampler):
                if idx.numel() == B:
                    if graphed.enabled and graphed.graph is None:
                        # (every tensor a step updates: incl. the optimizer-written bf16 FC shadow and
                        # the BN batch counters)
                        _capture_preserving(graphed, state(), static_idx, idx)
                    static_idx.copy_(idx)
                    graphed()
                else:
                    run(idx)
                nb += 1
                if it % self.print_freq == 0:
                    l = last_loss.tolist()
                    self._print(f"Epoch: [{epoch}/{self.n_epochs}][{it}/{len(sampler)}]\t Loss {l[0]:.5f}\t "
                                f"Loss_perf {l[1]:.5f}")
            if ctx.device.type == "cuda":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            sps = nb * B * E * U * (1 if ref else ctx.world) / max(dt, 1e-9)
            # the epoch's loss over every rank: reference semantics -- shares of one loss (sum); weak -- mean
            ctx.all_reduce_(loss_acc)
            tl = (loss_acc / (max(nb, 1) * (1 if ref else ctx.world))).tolist()
            ctx.heartbeat(f"hdce epoch {epoch}: validation")   # (failure detector: a sync point completed)
            self.train_HDCE_losses.append(tl[0])
            self._sync_bn_buffers(model)
            nmse, nmse_perf = self.eval_hdce(model, va)
            self.val_HDCE_nmse.append(nmse)
            if ctx.is_main:
                with disarmed("hdce checkpoint"):
                    if epoch == self.n_epochs - 1:
                        ck.save_hdce(d, model.convs, model.fc, B, self.SNRdb, f"epoch{epoch}")
                        print("HDCE finally saved!")
                    if nmse < best_nmse:
                        ck.save_hdce(d, model.convs, model.fc, B, self.SNRdb, "best")
                        print("HDCE saved!")
            if nmse < best_nmse:
                best_nmse = nmse
            self._print(f"Epoch [{epoch}]/[{self.n_epochs}] || NMSE {nmse:.5f}, NMSE_perf {nmse_perf:.5f}, "
                        f"best nmse: {best_nmse:.5f}")
            self._print("==============================================================")
            log.log(kind="hdce_epoch", epoch=epoch, loss=tl[0], loss_perf=tl[1], val_nmse=nmse,
                    val_nmse_db=to_db(nmse), val_nmse_perf_db=to_db(nmse_perf), lr=opt.lr, samples_per_sec=sps,
                    fc_path=getattr(step, "fc_path", None), f8_bwd=bool(getattr(step, "_f8_bwd", False)))
            if swa is not None and epoch >= self.n_epochs - self.swa_epochs:
                swa[0].add_(sp.flat)
                swa[1] += 1
            if epoch > 0:
                if epoch % self.lr_decay == 0:
                    opt.set_lr(opt.lr * 0.5)
                if opt.lr < self.lr_threshold:
                    opt.set_lr(self.lr_threshold)
            if ctx.is_main:
                with disarmed("hdce resume file"):
                    ck.save_resume(resume_path, epoch=epoch, best=best_nmse, optimizer=opt.state_dict(),
                                   flat=sp.flat.cpu(), run_mean=[t.cpu() for t in model.run_mean],
                                   run_var=[t.cpu() for t in model.run_var], nbt=[t.cpu() for t in model.nbt],
                                   train_losses=torch.tensor(self.train_HDCE_losses, dtype=torch.float64),
                                   val_nmse=torch.tensor(self.val_HDCE_nmse, dtype=torch.float64),
                                   rng=ck.rng_state(),
                                   **({"swa": swa[0].cpu(), "swa_n": swa[1]} if swa is not None else {}))
            ctx.heartbeat(f"hdce epoch {epoch + 1}")
            _maybe_fault(epoch)
        if swa is not None and swa[1] > 0 and ctx.is_main:
            with disarmed("hdce swa (rank 0)"):
                self._save_swa(model, tr, swa, d)
            ctx.heartbeat("hdce swa")
        self.hdce_model = model
        return model

    @torch.no_grad()
    def _save_swa(self, model: HDCEModel, store: DMLStore, swa: list, d: str) -> None:
        """``swa_epochs``: the mean of the last epochs' weight snapshots, with every expert's BN statistics
        re-estimated on its own training streams -- torch's momentum=None cumulative average over batches of
        n_users x batch_size_DML samples, the training step's BN batch (the running statistics of the trained
        weights do not describe the averaged ones) -- saved under the tag "swa" for ``model_val(hdce_tag="swa")``.
        The trained weights and statistics are put back afterwards.  (An estimator-side option beside the
        reference protocol, which evaluates the last epoch: Test.py:64-100.  Data parallel: rank 0 re-estimates the
        statistics on its own training shard -- every rank holds the same averaged weights -- and saves.)"""
        from .evaluate import recalibrate_bn, restore_bn
        sp = model.space
        keep = sp.flat.clone()
        sp.flat.copy_(swa[0] / swa[1])
        xs, ex = [], []
        for e in range(self.n_scenarios):
            streams = (store.scen == e).nonzero().flatten().to(store.Yp.device)
            Yp = store.Yp.index_select(0, streams)               # (U, n, ...): sample-major, the users of one
            xs.append(Yp.transpose(0, 1).reshape(-1, *Yp.shape[2:]))   # index next to each other, as in a batch
            ex.append(torch.full((xs[-1].shape[0],), e, dtype=torch.int64, device=store.Yp.device))
        x, expert = torch.cat(xs), torch.cat(ex)
        chunk = self.n_users * self.batch_size_DML
        if store.Yp.is_cuda and self.hdce_engine == "hip":
            from .infer import HIPInference
            eng = HIPInference(model.convs, model.fc, self.Pilot_num, store.Yp.device)
            saved = eng.recalibrate_bn(model.convs, x, expert, chunk=chunk)
        else:
            saved = recalibrate_bn(model.convs, x, expert, chunk=chunk)
        ck.save_hdce(d, model.convs, model.fc, self.batch_size_DML, self.SNRdb, "swa")
        restore_bn(model.convs, saved)
        sp.flat.copy_(keep)
        self._print(f"HDCE weight average over {swa[1]} epochs saved (tag swa)")

    # ------------------------------------------------------------------ classifiers
    @torch.no_grad()
    def eval_classifier(self, cstep: ClassifierStep, store: DMLStore, batch: int) -> Tuple[float, float]:
        """(avg val loss, accuracy) with the reference's definitions (R:378-414)."""
        model = cstep.model
        model.eval()
        S = store.n_streams
        loss_sum = torch.zeros(4, device=store.Yp.device, dtype=torch.float64)  # loss sum, correct, total, batches
        nb = 0
        for s in range(0, store.n, batch):
            idx = torch.arange(s, min(s + batch, store.n), device=store.Yp.device)
            b = idx.numel()
            x = store.Yp.index_select(1, idx).reshape(S * b, *store.Yp.shape[2:])
            labels = store.scen.repeat_interleave(b)
            out = cstep.forward(x)
            loss_sum[0] += F.nll_loss(out, labels).double()
            loss_sum[1] += (out.argmax(1) == labels).sum().double()
            loss_sum[2] += labels.numel()
            nb += 1
        ctx = self._context()
        loss_sum[3] = nb
        ctx.all_reduce_(loss_sum)   # (per-rank val shards may differ in size: divide global sums)
        loss_sum[0] /= loss_sum[3].clamp_min(1)
        model.train()
        out = float(loss_sum[0]), float(loss_sum[1] / loss_sum[2])
        ctx.heartbeat()
        return out

    def _train_classifier(self, model, kind: str, opt_name: str, wd: float, prune_thr: float,
                          on_epoch, histories: Tuple[List, List, List], extra: Optional[Dict] = None):
        """``extra``: small mutable trainer state (e.g. best accuracy) saved in the resume file."""
        ctx = self._context()
        tr, va = self.device_stores()
        model = model.to(ctx.device)
        space = FlatParamSpace(list(model.named_parameters()), ctx.device)
        ctx.broadcast_(space.flat)
        kw = {"prune_thr": prune_thr}
        if opt_name == "adamw":
            kw["weight_decay"] = wd
        opt = make_optimizer(space, opt_name, self.lr, **kw)
        S, B = tr.n_streams, self.batch_size_DML
        ref = self._dp_reference()
        Bl = (B + ctx.world - 1) // ctx.world if ref else B
        cstep = ClassifierStep(model, S, space=space, batch_total=S * Bl)
        skip = cstep.skip if self.nan_guard else None
        buckets = GradBuckets(ctx, {"all": [space.grad] + ([skip] if skip is not None else [])})
        cstep.grad_hook = buckets.launch
        loss_acc = torch.zeros(1, device=ctx.device)
        static_idx = torch.zeros(B, dtype=torch.long, device=ctx.device)
        gscale = 1.0 / ctx.world

        def run(idx):
            space.zero_grad()
            if ref:   # (mean NLL of the global batch = sum over ranks of (n_r / n) x the rank's mean)
                n_glob = idx.numel()
                idx = self._local_part(idx)
                share = idx.numel() * ctx.world / n_glob
                if share != 1.0:
                    cstep.grad_hook = None
            b = idx.numel()
            if b == 0:
                # a partial last batch smaller than the world: no rows here, but every collective and the
                # optimizer step still run in lockstep (zero gradients, a clear NaN flag)
                if skip is not None:
                    skip.zero_()
                cstep.grad_hook = buckets.launch
                buckets.launch_all()
                buckets.wait()
                opt.step(grad_scale=gscale, skip=skip)
                return
            x = tr.Yp.index_select(1, idx).reshape(S * b, *tr.Yp.shape[2:])
            labels = tr.scen.repeat_interleave(b)
            loss = cstep(x, labels)
            if ref and share != 1.0:   # (uneven parts: weight this rank's mean before the reduction)
                space.grad.mul_(share)
                loss = loss * share
                cstep.grad_hook = buckets.launch
                buckets.launch_all()
            loss_acc.add_(loss)
            buckets.wait()
            opt.step(grad_scale=gscale, skip=skip)

        graphed = GraphedStep(lambda: run(static_idx), enabled=self._graphs_on())
        sampler = DeviceSampler(tr.n, B, ctx.device, self.seed + 17, 0 if ref else ctx.rank)
        log = self._log()
        train_losses, val_losses, val_accs = histories
        for h in histories:
            h.clear()
        extra = extra if extra is not None else {}
        resume_path = os.path.join(ck.ckpt_dir(self.workspace, self.Pilot_num),
                                   f"{kind.upper()}_{B}_{self.SNRdb}dB_resume.pth")
        start = 0
        if self.resume:
            st = ck.load_resume(resume_path)
            if st is not None:
                ck.load_into(space.flat, st["flat"])
                opt.load_state_dict(st["optimizer"])
                for h, v in zip(histories, st["histories"]):
                    h.extend(v.tolist())
                extra.update({k: float(v) for k, v in st["extra"].items()})
                start = int(st["epoch"]) + 1
                if ctx.world == 1:
                    ck.set_rng_state(st["rng"])
                self._print(f"Resumed {kind.upper()} from {resume_path} at epoch {start}")
        for epoch in range(start, self.n_epochs):
            model.train()
            sampler.set_epoch(epoch)
            loss_acc.zero_()
            opt.pruned.zero_()
            nb = 0
            t0 = time.perf_counter()
            for idx in sampler:
                if idx.numel() == B:
                    if graphed.enabled and graphed.graph is None:
                        _capture_preserving(graphed, [space.flat, opt.step_t, loss_acc, opt.pruned]
                                            + ([opt.m, opt.v] if opt.kind != "sgd" else [opt.buf])
                                            + ([cstep.hip.noise_ctr] if getattr(cstep.hip, "noise_ctr", None)
                                               is not None else []),
                                            static_idx, idx)
                    static_idx.copy_(idx)
                    graphed()
                else:
                    run(idx)
                nb += 1
            ctx.all_reduce_(loss_acc)   # (the epoch's mean loss over every rank)
            avg = float(loss_acc.item()) / (max(nb, 1) * ctx.world)
            ctx.heartbeat(f"{kind} epoch {epoch}: validation")
            dt = time.perf_counter() - t0
            train_losses.append(avg)
            self._print(f"Epoch {epoch + 1}/{self.n_epochs}, Average Loss: {avg:.4f}")
            if prune_thr > 0:
                ratio = opt.pruning_ratio(nb)
                if ratio > 0.1:
                    self._print(f"Gradient pruning: {ratio:.1%} gradients pruned")
            vl, acc = self.eval_classifier(cstep, va, B)
            val_losses.append(vl)
            val_accs.append(acc)
            self._print(f"Validation Loss: {vl:.4f}, Validation Accuracy: {acc:.2%}")
            log.log(kind=f"{kind}_epoch", epoch=epoch, loss=avg, val_loss=vl, val_acc=acc, lr=opt.lr,
                    samples_per_sec=nb * B * S * ctx.world / max(dt, 1e-9))
            on_epoch(epoch, acc, model)
            if ctx.is_main:
                ck.save_resume(resume_path, epoch=epoch, flat=space.flat.cpu(), optimizer=opt.state_dict(),
                               histories=[torch.tensor(h, dtype=torch.float64) for h in histories],
                               extra={k: torch.tensor(float(v)) for k, v in extra.items()}, rng=ck.rng_state())
            _maybe_fault(epoch)
        return model

    def train_QSC_P128(self):
        self._sync_cfg()
        self._context()  # seeds before the model is built
        model = QSC_P128(self.n_qubits, self.n_layers, self.n_classes, use_quantumnat=self.use_quantumnat,
                         use_gradient_pruning=self.use_gradient_pruning, pilot_num=self.Pilot_num,
                         backend=None if self.backend == "auto" else self.backend, noise_level=self.noise_level,
                         gradient_threshold=self.gradient_threshold)
        ctx = self._context()
        d = ck.ckpt_dir(self.workspace, self.Pilot_num) if ctx.is_main else None
        state = {"best": 0.0}
        self._print("Data Loaded for QSC with QuantumNAT + On-chip QNN optimization!")

        def on_epoch(epoch, acc, m):
            if ctx.is_main and acc > state["best"]:
                ck.save_qsc(d, m, self.batch_size_DML, self.SNRdb, "best", alias=True)
                print("Optimized QML saved (best so far).")
            if acc > state["best"]:
                state["best"] = acc
            if ctx.is_main and epoch == self.n_epochs - 1:
                ck.save_qsc(d, m, self.batch_size_DML, self.SNRdb, f"epoch{epoch}")
                print("Optimized QSC finally saved!")

        prune = self.gradient_threshold if self.use_gradient_pruning else 0.0
        self.qsc_model = self._train_classifier(model, "qsc", "adamw", self.qsc_weight_decay, prune, on_epoch,
                                                (self.train_QSC_losses, self.val_QSC_losses, self.val_QSC_accuracies),
                                                extra=state)
        return self.qsc_model

    def train_SC_P128(self):
        """Classical scenario classifier trainer (Test.py:69-73 expects its checkpoint)."""
        self._sync_cfg()
        self._context()
        model = SC_P128(self.Pilot_num, self.n_classes)
        ctx = self._context()
        d = ck.ckpt_dir(self.workspace, self.Pilot_num) if ctx.is_main else None
        self.val_SC_losses, self.val_SC_accuracies = [], []

        def on_epoch(epoch, acc, m):
            if ctx.is_main and epoch == self.n_epochs - 1:
                ck.save_sc(d, m, self.batch_size_DML, self.SNRdb, f"epoch{epoch}")
                print("SC finally saved!")

        self.sc_model = self._train_classifier(model, "sc", self.optimizer, 0.0, 0.0, on_epoch,
                                               (self.train_SC_losses, self.val_SC_losses, self.val_SC_accuracies))
        return self.sc_model

    def train_all(self):
        """HDCE estimator + classical SC + quantum SC: everything model_val needs."""
        self.train_Conv_Linear_of_HDCE()
        self.train_SC_P128()
        self.train_QSC_P128()


def _maybe_fault(epoch: int) -> None:
    """Fault injection for the resume tests: QDML_FAULT_EPOCH=k hard-kills the process right after
    epoch k's resume file is written (no cleanup, like a node loss)."""
    k = os.environ.get("QDML_FAULT_EPOCH")
    if k is not None and int(k) == epoch:
        print(f"[fault injection] killing the process after epoch {epoch}", flush=True)
        os._exit(75)


def _capture_preserving(graphed: GraphedStep, state: List[torch.Tensor], static_idx: torch.Tensor,
                        idx: torch.Tensor) -> None:
    """Capture the step graph without letting the warm-up iterations change training state:
    snapshot every stateful tensor, warm up + capture, restore."""
    snap = [t.clone() for t in state]
    static_idx.copy_(idx)
    graphed.capture()
    with torch.no_grad():
        for t, s in zip(state, snap):
            t.copy_(s)
