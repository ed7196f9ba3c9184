"""Device-resident, hipGraph-captured Wide&Deep trainer on the fused gfx950 kernels.

One training step = ``wdc_fused`` (csrc/wd_chain.hip; or ``wd_fused`` with kernel="tile") (forward + loss +
backward, per-workgroup gradient slabs) -> ``wd_reduce_opt`` (full slab sum + Adagrad/FTRL/Adam/SGD + bf16 weight image in ONE launch). When
data-parallel the local sum is written to ONE flat 82 KB gradient bucket, RCCL all-reduced over xGMI,
and the optimizer launch reads that bucket. (The older two-launch ``wd_reduce`` -> ``wd_optimizer``
path stays selectable with ``fused_update=False`` for A/B.) The input
shard lives in HBM; the data offset advances through a device-side step counter, so the whole
step (collective included) can be captured once and replayed as a hipGraph.

Reference behaviour: Estimator train loop of `taxi_utils.py:285-356` (read_batch_features ->
DNNLinearCombinedClassifier step with FTRL + Adagrad).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import os

import numpy as np
import torch

from ..models import wide_deep as wdm
from ..ops import wide_deep as wdk

OPT_KIND = {"sgd": 0, "adagrad": 1, "ftrl": 2, "adam": 3}


@dataclass
class OptSpec:
    kind: str = "adagrad"
    lr: float = 0.05
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    l1: float = 0.0
    l2: float = 0.0
    lr_power: float = -0.5
    initial_accumulator_value: float = 0.1

    def encode(self) -> torch.Tensor:
        return torch.tensor([OPT_KIND[self.kind], self.lr, self.beta1, self.beta2, self.eps, self.l1, self.l2,
                             self.lr_power], dtype=torch.float32)


def default_dnn_opt() -> OptSpec:
    return OptSpec("adagrad", lr=0.05)


def default_wide_opt(num_linear_columns: int = 9) -> OptSpec:
    return OptSpec("ftrl", lr=min(0.2, 1.0 / math.sqrt(num_linear_columns)))


class FusedWideDeepTrainer:
    """kernel="chain" (default): csrc/wd_chain.hip, register-chained MFMA forward/backward, 128 examples per
    workgroup iteration; kernel="tile": csrc/wide_deep.hip (wd_fused), LDS-staged activations, 64 per tile.
    Both write the same kind of per-workgroup gradient slab, reduced + applied by wd_reduce_opt."""

    def __init__(self, model: wdm.WideDeepModel | None = None, batch: int = 40, device="cuda",
                 dnn_opt: OptSpec | None = None, wide_opt: OptSpec | None = None, loss_reduction: str = "sum",
                 grid: int | None = None, process_group=None, max_grid: int = 256, compact_slab: bool = True,
                 live_staging: bool = False, fused_update: bool = True, kernel: str = "chain", waves: int = 8,
                 in_kernel_tail: bool | None = None, persistent: bool | None = None, one_launch: bool | None = None,
                 small_tile: bool | None = None, shuffle_seed: int = 0, feed_stride: int | None = None,
                 feed_offset: int = 0, large_tile: bool | None = None):
        """shuffle_seed: 0 trains on the records in stored order; any other value draws a fresh pseudo-random
        permutation of the resident records every epoch inside the kernel's record fetch (csrc/feed.h; the
        reference's `read_batch_features(randomize_input=True)`, `taxi_utils.py:275-276`). feed_stride / feed_offset:
        this replica's place in a global record stream shared by data-parallel ranks (stride = world x batch,
        offset = rank x batch; default: its own stream, stride = batch, offset 0)."""
        self.device = torch.device(device)
        self.model = model or wdm.WideDeepModel()
        wdm.check_fused_compatible(self.model.cfg)
        if kernel not in ("chain", "tile"):
            raise ValueError("kernel must be 'chain' or 'tile'")
        self.kernel = kernel
        self.waves = int(waves)  # chained kernel: 8 (2 waves / SIMD x 16 examples) or 4 (1 wave / SIMD x 32)
        c = wdk.constants()
        assert c["WTOT"] == wdm.WTOT and c["STRIDE"] == wdm.STRIDE and c["NWIDE"] == wdm.NWIDE
        if kernel == "chain":
            from ..ops import wd_chain as wdc

            cc = wdc.constants()
            assert cc["LWEND"] == wdm.CHAIN_LWEND and cc["PAD"] == wdm.CHAIN_PAD
            if not fused_update or not compact_slab or live_staging:
                raise ValueError("the chained kernel uses the compact slab, full staging and the fused update")
            self.T = cc["T"]
        else:
            self.T = c["T"]
        self.batch = int(batch)
        self.shuffle_seed = int(shuffle_seed)
        self.feed_stride = int(feed_stride) if feed_stride is not None else self.batch
        self.feed_offset = int(feed_offset)
        if not (self.feed_stride >= self.batch and 0 <= self.feed_offset <= self.feed_stride - self.batch):
            raise ValueError("need feed_stride >= batch and 0 <= feed_offset <= feed_stride - batch")
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        ntiles = (self.batch + self.T - 1) // self.T
        self.grid = int(grid or min(ntiles, max_grid))
        # large batches (more than one T = 128 iteration per workgroup): the T = 256 build, one iteration of 256
        # examples per workgroup (csrc/wd_chain256.hip; MIFX_WD_T256=0 or large_tile=False turns it off)
        if large_tile is None:
            large_tile = os.environ.get("MIFX_WD_T256", "1") == "1"
        tail_req = in_kernel_tail if in_kernel_tail is not None else os.environ.get("MIFX_WD_TAIL", "0") == "1"
        self._t256 = bool(large_tile and kernel == "chain" and self.waves == 8 and grid is None and not tail_req
                          and ntiles > max_grid and (self.batch + 255) // 256 <= max_grid)
        if self._t256:
            self.grid = (self.batch + 255) // 256
        self.dnn_opt = dnn_opt or default_dnn_opt()
        self.wide_opt = wide_opt or default_wide_opt(len(self.model.cfg.wide))
        self.loss_reduction = loss_reduction
        dev = self.device
        # compact_slab: store/reduce/all-reduce only the dW tiles that hold trainable entries;
        # live_staging: stage only the live rows/granules of the weight image into LDS
        if kernel == "chain":
            tmap, self.stride, gidx, mask, wmap = wdm.chain_maps(self.model.cfg)
            self.wmap = torch.from_numpy(wmap).to(dev)
        else:
            gidx, mask = wdm.canonical_index_maps(self.model.cfg, compact_slab)
            tmap, self.stride = wdm.compact_tile_map(self.model.cfg, compact_slab)
            self.wmap = None
        self.gidx_np = gidx
        self.stage_dims = wdm.stage_dims(self.model.cfg) if live_staging else None
        self.tmap = torch.from_numpy(tmap).to(dev)
        self.gidx = torch.from_numpy(gidx).to(dev)
        self.mask = torch.from_numpy(mask).to(dev)
        param = torch.from_numpy(wdm.pack_canonical(self.model)).to(dev)
        n = wdm.WTOT + wdm.NWIDE
        s0 = torch.zeros(n, device=dev)
        s1 = torch.zeros(n, device=dev)
        for sl, spec in ((slice(0, wdm.WTOT), self.dnn_opt), (slice(wdm.WTOT, n), self.wide_opt)):
            if spec.kind in ("adagrad", "ftrl"):
                s0[sl] = spec.initial_accumulator_value
        # inverse of the (bijective on live entries) canonical -> slab-column map, -1 on padding columns
        inv = np.full(self.stride, -1, dtype=np.int32)
        live = np.nonzero(mask)[0]
        inv[gidx[live]] = live.astype(np.int32)
        self.inv = torch.from_numpy(inv).to(dev)
        # Chained kernel: the master weights and optimizer state live in SLAB-COLUMN order (param_sc / s0_sc /
        # s1_sc [stride]) so the optimizer kernels index them by the gradient's own column (no inv[] -> state ->
        # wmap chain of dependent loads; csrc/wide_deep.hip wd_reduce_opt_sc). wsc[col]: -1 padding, -2 wide
        # weight, >= 0 DNN weight with its bf16 weight-image offset. `param` / `s0` / `s1` are canonical views.
        self._sc = kernel == "chain"
        self._gidx_l = self.gidx.long()
        self._mask_b = self.mask.bool()
        if self._sc:
            wsc = np.full(self.stride, -1, dtype=np.int32)
            dnn_live = live[live < wdm.WTOT]
            wsc[gidx[dnn_live]] = wmap[dnn_live]
            wsc[gidx[live[live >= wdm.WTOT]]] = -2
            self.wsc = torch.from_numpy(wsc).to(dev)
            self._frozen = tuple(torch.where(self._mask_b, torch.zeros_like(v), v) for v in (param, s0, s1))
            self.param_sc, self.s0_sc, self.s1_sc = (self._to_sc(v) for v in (param, s0, s1))
        else:
            self._param, self._s0, self._s1 = param, s0, s1
        self.wt = self._weight_image()
        self.fused_update = bool(fused_update)
        # per-optimizer-workgroup step slots (slot 0 = the step; see csrc/wide_deep.hip STEP_SLOTS)
        self.step_ctr = torch.zeros(wdk.STEP_SLOTS, dtype=torch.int64, device=dev)
        self.slab = torch.empty(self.grid, self.stride, device=dev)
        # chained kernel, one rank: XCD-local two-level slab reduction (each XCD's slab rows summed where its L2
        # holds them; csrc/wide_deep.hip wd_reduce_xcd)
        # (small grids keep the one-pass reduce: below ~64 workgroups there is little slab to keep local)
        # default: the residue-class variant (rows b == k mod 8 per partial; no placement record, no XCD ordering:
        # csrc/wide_deep.hip wd_reduce_res) -- 29.9 vs 32.4 us per headline step on MI355X
        # (profiles/wd_res_ab_r6.jsonl); MIFX_WD_RES=0: the placement-recorded XCD reduction
        use_xcd = os.environ.get("MIFX_WD_XCD", "1") != "0"
        # (data parallelism keeps the XCD-recorded scratch: the xGMI exchange kernel sums the per-XCD partials itself,
        # mifx.parallel.xgmi.XgmiExchange.reduce_apply)
        red_cls = wdk.ResReduce if os.environ.get("MIFX_WD_RES", "1") == "1" and self.world == 1 else wdk.XcdReduce
        self._xcd = red_cls(self.stride, dev) if use_xcd and self._sc and 64 <= self.grid <= 256 else None
        # in_kernel_tail=True (or MIFX_WD_TAIL=1): the whole step in ONE launch -- slab reduction + optimizer inside
        # the fused kernel after two grid-wide barriers (csrc/wd_chain.hip TailArgs; needs every workgroup resident:
        # grid <= #CUs, one workgroup per CU by its LDS). Measured SLOWER on MI355X and therefore off by default:
        # 40.8 vs 33.6 us per step at B=65536 (profiles/archive/wd_tail_ab_r3.md): each cross-XCD grid barrier costs ~3 us
        # (arrival atomic + polling through the fabric) and the write-through per-XCD partials ~7 us more before
        # the second barrier, against ~11.6 us for the two tail kernels they replace.
        if in_kernel_tail is None:
            in_kernel_tail = os.environ.get("MIFX_WD_TAIL", "0") == "1"
        self._ktail = None
        if in_kernel_tail and self._sc and self.world == 1 and 64 <= self.grid <= 256 and self.waves == 8 \
                and self.device.type == "cuda" and self.grid <= torch.cuda.get_device_properties(dev).multi_processor_count:
            from ..ops import wd_chain as wdc

            self._ktail = wdc.InKernelTail(self.stride, dev)
        # persistent (opt-in: persistent=True or MIFX_WD_PERSIST=1; one rank, batch <= T): run(n) is ONE launch of
        # one workgroup doing n whole steps -- the weight image stays in LDS across them and the optimizer runs in
        # the workgroup (csrc/wd_chain.hip opt_tiles / mifx_wdc_persist); bit-identical to the slab path. Measured
        # SLOWER on MI355X at B=40: 25.6 us/step vs 14.8 us for the two-kernel graph step (profiles/
        # wd_persist_ab_r3.md): the optimizer's ~750 KB of master-state traffic per step through ONE CU's memory
        # path costs more than the 370-workgroup optimizer launch plus the weight re-staging it saves.
        if persistent is None:
            persistent = os.environ.get("MIFX_WD_PERSIST", "0") == "1"
        self._persist = bool(persistent and self._sc and self.world == 1 and self.grid == 1 and self.batch <= self.T
                             and self.waves == 8 and self._ktail is None and self.device.type == "cuda")
        # small_tile (default on; small_tile=False or MIFX_WD_T64=0 turns it off): a batch of <= 64 examples trains
        # on the T = 64 build of the chained kernel (csrc/wd_chain64.hip: one 4-wave workgroup, one wave per SIMD)
        # instead of one 8-wave T = 128 iteration that is mostly padding at the reference batch of 40
        if small_tile is None:
            small_tile = os.environ.get("MIFX_WD_T64", "1") == "1"
        self.tile = 256 if self._t256 else 64 if (small_tile and kernel == "chain" and self.batch <= 64 and self.grid == 1
                                                  and not self._persist and self._ktail is None) else 128
        if self.tile == 64:
            self.waves = 4
        # one launch per step when ONE workgroup trains the batch (opt-in: one_launch=True or MIFX_WD_ONE_LAUNCH=1;
        # grid 1, one rank): the optimizer runs in extra workgroups of the fused launch, which load their columns'
        # state during the step and update once workgroup 0 has published the gradient row (csrc/wd_chain.hip
        # help_update), instead of in a second kernel after it. Bit-identical to the two-kernel step (wd_opt1_sc's
        # partition and step slots). Measured at the reference batch of 40: 13.55 vs 13.25 us per step
        # (profiles/wd_one_launch_ab_r4.txt; 17.6 with acquire-ordered polls, which invalidate L2 on every poll) --
        # the flag poll and the cache-bypassing read of the row after it cost what the saved launch did.
        if one_launch is None:
            one_launch = os.environ.get("MIFX_WD_ONE_LAUNCH", "0") == "1"
        self._one = None
        if one_launch and self._sc and self.world == 1 and self.grid == 1 and self.fused_update \
                and not self._persist and self._ktail is None and self.device.type == "cuda" \
                and (self.tile == 64 or (self.tile == 128 and self.waves == 8)):
            from ..ops import wd_chain as wdc

            self._one = wdc.OneRowTail(self.stride, self.tile, dev)
        self.slab_loss = torch.zeros(self.grid, device=dev)
        self.nsplit = max(1, min(16, self.grid // 8))
        self.partial = torch.empty(self.nsplit, self.stride, device=dev)
        self.grad = torch.empty(1, self.stride, device=dev)  # the DP all-reduce payload (compact)
        self.h_dnn = self.dnn_opt.encode()
        self.h_wide = self.wide_opt.encode()
        self.records = None
        self.n_data = 0
        self.graph = None
        self._graphs = None
        self._fast = None
        self._direct = None
        self._xg = None  # xGMI gradient exchange (enable_xgmi)
        self.graph_multi, self.graph_multi_steps = None, 1

    # ---------------------------------------------------------------- master state views
    def _to_sc(self, v: torch.Tensor) -> torch.Tensor:
        out = torch.zeros(self.stride, device=self.device)
        out[self._gidx_l[self._mask_b]] = v.to(self.device)[self._mask_b]
        return out

    def _canon(self, v_sc: torch.Tensor, frozen: torch.Tensor) -> torch.Tensor:
        return torch.where(self._mask_b, v_sc[self._gidx_l], frozen)

    @property
    def param(self) -> torch.Tensor:
        """fp32 master weights in canonical order [WTOT + NWIDE] (a copy for the chained kernel)."""
        return self._canon(self.param_sc, self._frozen[0]) if self._sc else self._param

    @property
    def s0(self) -> torch.Tensor:
        return self._canon(self.s0_sc, self._frozen[1]) if self._sc else self._s0

    @property
    def s1(self) -> torch.Tensor:
        return self._canon(self.s1_sc, self._frozen[2]) if self._sc else self._s1

    def set_master_state(self, param=None, s0=None, s1=None) -> None:
        """Overwrite weights / optimizer state (canonical order); re-emits the bf16 weight image."""
        for i, (name, v) in enumerate((("param", param), ("s0", s0), ("s1", s1))):
            if v is None:
                continue
            v = torch.as_tensor(v, dtype=torch.float32).to(self.device)
            if self._sc:
                getattr(self, name + "_sc").copy_(self._to_sc(v))
                fr = list(self._frozen)
                fr[i] = torch.where(self._mask_b, torch.zeros_like(v), v)
                self._frozen = tuple(fr)
            else:
                getattr(self, "_" + name).copy_(v)
        if param is not None:
            self.wt.copy_(self._weight_image())

    @property
    def wide_weights(self) -> torch.Tensor:
        """The wide (linear) weights the fused kernel reads, canonical order [NWIDE] (a view)."""
        if self._sc:
            w0 = self.stride - wdm.WIDE_PAD
            return self.param_sc[w0:w0 + wdm.NWIDE]
        return self._param[wdm.WTOT:]

    def _weight_image(self) -> torch.Tensor:
        """bf16 (as int16) weight image the fused kernel stages: canonical order (tile kernel) or the chained
        kernel's C-ordered LDS layout."""
        if self.kernel == "chain":
            img = torch.from_numpy(wdm.chain_image(self.param.cpu()))
            return img.to(self.device).to(torch.bfloat16).view(torch.int16).contiguous()
        return self.param[: wdm.WTOT].to(torch.bfloat16).view(torch.int16).contiguous()

    def feed_args(self) -> tuple[int, int, int]:
        """(stride, offset, shuffle key) of the training record stream (csrc/feed.h)."""
        return self.feed_stride, self.feed_offset, self.shuffle_seed & (2**64 - 1)

    def _launch(self, records, n, batch, start_fixed, step_ctr, slab, slab_loss, logits, grid, train) -> None:
        feed = self.feed_args() if train else None
        if self.kernel == "chain":
            from ..ops import wd_chain as wdc

            wdc.fused(records, n, batch, start_fixed, step_ctr, self.wt, self.wide_weights, slab, slab_loss,
                      logits, self.grad_scale, grid, train, self.tmap if train else None, self.waves,
                      self._xcd.xcd_of if (train and self._xcd is not None and slab is self.slab) else None,
                      tile=self.tile if train else 128, feed=feed)
        else:
            wdk.fused(records, n, batch, start_fixed, step_ctr, self.wt, self.wide_weights, slab, slab_loss,
                      logits, self.grad_scale if train else 1.0, grid, train, self.tmap if train else None,
                      self.stage_dims, feed=feed)

    # ---------------------------------------------------------------- data
    def set_data(self, records: torch.Tensor) -> None:
        """records: uint8 [N, 32] packed taxi records (see models.wide_deep.RECORD_DTYPE)."""
        if records.dim() != 2 or records.shape[1] != 32 or records.dtype != torch.uint8:
            raise ValueError("records must be uint8 [N, 32]")
        self.records = records.to(self.device).contiguous()
        self.n_data = self.records.shape[0]
        self.graph, self._graphs, self._fast = None, None, None
        self.graph_multi, self.graph_multi_steps = None, 1

    @property
    def grad_scale(self) -> float:
        if self.loss_reduction == "sum":
            return 1.0
        return 1.0 / (self.batch * self.world)

    # ---------------------------------------------------------------- step
    def _local_grad(self) -> None:
        """fused fwd/bwd + slab reduction; for world>1 the result lands in `self.grad` (one row)."""
        self._launch(self.records, self.n_data, self.batch, 0, self.step_ctr, self.slab, self.slab_loss, None,
                     self.grid, True)
        if self.fused_update:
            if self.world > 1:
                wdk.reduce_full(self.slab, self.grid, self.grad)
        elif self.world == 1:
            if self.grid > 1:
                wdk.reduce(self.slab, self.grid, self.nsplit, self.partial)
        elif self.grid == 1:
            self.grad.copy_(self.slab)
        else:
            wdk.reduce(self.slab, self.grid, self.nsplit, self.partial)
            wdk.reduce(self.partial, self.nsplit, 1, self.grad)

    def _apply(self) -> None:
        if self.fused_update:
            src, groups = (self.slab, self.grid) if self.world == 1 else (self.grad, 1)
            if self._sc and self.world == 1 and self._xcd is not None:
                self._xcd.apply_sc(self.slab, self.grid, self.wsc, self.param_sc, self.s0_sc, self.s1_sc, self.wt,
                                   self.step_ctr, self.h_dnn, self.h_wide)
            elif self._sc:
                wdk.reduce_apply_sc(src, groups, self.wsc, self.param_sc, self.s0_sc, self.s1_sc, self.wt,
                                    self.step_ctr, self.h_dnn, self.h_wide)
            else:
                wdk.reduce_apply(src, groups, self.inv, self._param, self._s0, self._s1, self.wt, self.step_ctr,
                                 self.h_dnn, self.h_wide, self.wmap)
            return
        if self.world == 1:
            src, nparts = (self.slab, 1) if self.grid == 1 else (self.partial, self.nsplit)
        else:
            src, nparts = self.grad, 1
        wdk.optimizer(src, nparts, self.gidx, self.mask, self._param, self._s0, self._s1, self.wt, self.step_ctr,
                      self.h_dnn, self.h_wide)

    def _allreduce(self) -> None:
        if self.world > 1:
            if self._direct is not None:
                self._direct()
            else:
                torch.distributed.all_reduce(self.grad, group=self.pg)

    # ---------------------------------------------------------------- eager data-parallel fast path
    def _prepare_direct(self) -> None:
        """Data-parallel step without graphs: the three kernel launches with their ctypes arguments built once
        and the all-reduce issued straight to RCCL on the same stream (mifx.parallel.rccl_direct). Stream order
        is the only synchronisation; no graph-launch bubbles, no ProcessGroupNCCL stream hops."""
        import ctypes

        from ..ops import wd_chain as wdc
        from ..parallel.rccl_direct import DirectAllReduce
        from ..ops._lib import ptr

        if self.kernel != "chain" or not self.fused_update:
            raise ValueError("the direct DP path needs the chained kernel and the fused update")
        self._direct = DirectAllReduce(self.grad, self.pg)
        stream = torch.cuda.current_stream(self.device)
        sh = ctypes.c_void_p(stream.cuda_stream)
        fused = (wdc.fns_for(self.tile)["fused_f"],
                 (ptr(self.records), self.n_data, self.batch, 0, ptr(self.step_ctr), ptr(self.wt),
                  ptr(self.wide_weights), ptr(self.slab), ptr(self.slab_loss), None, float(self.grad_scale),
                  int(self.grid), 1, ptr(self.tmap), int(self.stride), int(self.waves), None, *self.feed_args(), sh))
        ro = wdk._fns()["reduce_opt"]
        red = (ro, (ptr(self.slab), int(self.grid), int(self.stride), ptr(self.grad), None, None, None, None, None, None,
                    None, None, None, sh))
        hd = self.h_dnn.contiguous()
        hw = self.h_wide.contiguous()
        app = (wdk._fns()["reduce_opt_sc"], (ptr(self.grad), 1, int(self.stride), ptr(self.wsc), ptr(self.param_sc),
                                             ptr(self.s0_sc), ptr(self.s1_sc), ptr(self.wt), ptr(self.step_ctr),
                                             ptr(hd), ptr(hw), sh))
        wdk._check_step_ctr(self.step_ctr)
        self._fast = (stream, fused, red, app, hd, hw)

    def _step_direct(self) -> None:
        stream, fused, red, app = self._fast[:4]
        if torch.cuda.current_stream(self.device) != stream:
            self._prepare_direct()
            stream, fused, red, app = self._fast[:4]
        for fn, args in (fused, red):
            if fn(*args) != 0:
                raise RuntimeError("W&D kernel launch failed")
        self._direct(stream)
        if app[0](*app[1]) != 0:
            raise RuntimeError("W&D optimizer launch failed")

    def _step_impl(self) -> None:
        if self._persist:
            from ..ops import wd_chain as wdc

            wdc.persist_steps(self, 1)
            return
        if self._ktail is not None:  # one launch: fwd/bwd + slab reduction + optimizer
            self._ktail.step(self)
            return
        if self._one is not None:  # one launch: fwd/bwd of the one workgroup + the optimizer workgroups
            self._one.step(self)
            return
        if self._xg is not None:  # data parallel over xGMI: no host collective, graph-capturable
            self._launch(self.records, self.n_data, self.batch, 0, self.step_ctr, self.slab, self.slab_loss, None,
                         self.grid, True)
            self._xg.reduce_apply(self)
            return
        self._local_grad()
        self._allreduce()
        self._apply()

    # ---------------------------------------------------------------- data parallel over xGMI
    def enable_xgmi(self) -> None:
        """Switch the data-parallel step to the one-shot xGMI gradient exchange (mifx.parallel.xgmi): the
        peers' local gradients are read straight from their HBM and summed with the optimizer in one kernel,
        so the whole step (all ranks in lock-step through device-side epoch flags) captures into hipGraphs.
        Runs the exchange self-test first; raises if it fails."""
        if self.world <= 1:
            raise ValueError("enable_xgmi needs a process group with more than one rank")
        if self.kernel != "chain" or not self.fused_update:
            raise ValueError("the xGMI step needs the chained kernel and the fused update")
        from ..parallel.xgmi import XgmiExchange

        self.disable_xgmi()
        xg = XgmiExchange(self.stride, self.pg, self.device)
        try:
            xg.selftest()
        except Exception:
            xg.close()
            raise
        self._xg = xg
        self.graph, self._graphs, self._fast = None, None, None
        self.graph_multi, self.graph_multi_steps = None, 1

    def _align_ranks(self) -> None:
        """Before the first exchange steps: load the fused kernel's code object (its first launch pays a
        one-time module load that can skew ranks by seconds) and line the ranks up on a host barrier, so no rank
        spins on the device for a peer that is still initialising."""
        self.predict_logits(self.records[: min(self.n_data, self.T)])
        torch.cuda.synchronize(self.device)
        torch.distributed.barrier(group=self.pg)

    def _check_exchange(self) -> None:
        """Raise if the xGMI exchange timed out on this rank (the kernels then stopped updating: see
        csrc/wide_deep.hip xg_wait). Called at every host synchronisation point."""
        if self._xg is not None:
            self._xg.check()
        if self._ktail is not None:
            self._ktail.check()
        if getattr(self, "_one", None) is not None:
            self._one.check()

    def disable_xgmi(self) -> None:
        if self._xg is not None:
            self._xg.close()
            self._xg = None
            self.graph, self.graph_multi, self.graph_multi_steps = None, None, 1

    @property
    def dp_exchange(self) -> str | None:
        if self.world <= 1:
            return None
        if self._xg is not None:
            return "xgmi"
        return "rccl-direct" if self._fast is not None else "collective"

    def step(self) -> None:
        if self.records is None:
            raise RuntimeError("call set_data() first")
        if self.graph is not None:
            self.graph.replay()
        elif self._fast is not None:  # data-parallel eager path with the direct RCCL all-reduce
            self._step_direct()
        elif self._graphs is not None:  # split capture: eager collective between two graphs
            self._graphs[0].replay()
            self._allreduce()
            self._graphs[1].replay()
        else:
            self._step_impl()

    def run(self, n: int) -> None:
        """n training steps. With a multi-step graph (capture(steps_per_graph=S)) this replays it n // S times and
        the one-step graph n % S times: every step still runs its own kernels (the data offset and optimizer
        step advance through the device-side step counter), the host just launches once per S steps. Replaying
        one graph per step left ~8.7 us of idle GPU between steps on MI355X (the host-side launch of a replay
        costs more than the step's ~35 us of GPU work): tools/timeline.py, profiles/archive/wd_step_timeline_r2.txt."""
        if self._persist:  # all n steps in one launch of the persistent kernel
            if n > 0:
                if self.records is None:
                    raise RuntimeError("call set_data() first")
                from ..ops import wd_chain as wdc

                wdc.persist_steps(self, n)
            return
        if self.graph_multi is not None and n >= self.graph_multi_steps:
            reps, n = divmod(n, self.graph_multi_steps)
            for _ in range(reps):
                self.graph_multi.replay()
        for _ in range(n):
            self.step()

    def capture(self, warmup: int = 2, include_collective: bool = False, steps_per_graph: int = 1,
                dp_mode: str = "direct") -> None:
        """Capture the step as hipGraph(s) after `warmup` eager steps on a side stream.

        Single rank: one graph (plus an S-step graph when steps_per_graph > 1). Multi-rank over RCCL, default
        (dp_mode="direct"): no graphs -- the fused, reduce and optimizer kernels launched eagerly from prebuilt
        ctypes arguments with the gradient all-reduce issued directly to RCCL in between, on the same stream
        (tools/dp_step_overhead.py). dp_mode="split": two graphs (local grad, optimizer) with the all-reduce
        issued eagerly between them (works with any backend, e.g. gloo); `include_collective=True`
        captures the RCCL all-reduce too -- one graph launch per step (bench.py --capture-collective; opt-in
        until validated on a multi-GPU node). On one MI355X with the DP path forced (tools/dp_step_overhead.py)
        the split-phase step costs 67.4 us vs 51.2 us captured at B=65536 (host 41.6 vs 11.4 us per step)."""
        if dp_mode == "xgmi" and self.world > 1 and self._xg is None:
            self.enable_xgmi()
        if self._xg is not None:
            self._align_ranks()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._step_impl()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graph, self._graphs, self._fast = None, None, None
        self.graph_multi, self.graph_multi_steps = None, 1
        if self.world == 1 or include_collective or self._xg is not None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step_impl()
            self.graph = g
            if steps_per_graph > 1 and not self._persist:  # S consecutive steps in one graph (see run())
                gm = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gm):
                    for _ in range(steps_per_graph):
                        self._step_impl()
                self.graph_multi, self.graph_multi_steps = gm, int(steps_per_graph)
            return
        if dp_mode == "direct" and self.kernel == "chain" and self.fused_update \
                and torch.distributed.get_backend(self.pg) == "nccl":
            self._prepare_direct()  # no graphs: eager launches + direct RCCL in stream order
            return
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            self._local_grad()
        with torch.cuda.graph(g2):
            self._apply()
        self._graphs = (g1, g2)

    # ---------------------------------------------------------------- introspection
    def last_loss(self) -> float:
        """Sum of per-example losses of the most recent step on this rank."""
        v = float(self.slab_loss.sum().item())
        self._check_exchange()
        return v

    @property
    def steps_done(self) -> int:
        v = int(self.step_ctr[0].item())
        self._check_exchange()
        return v

    def set_step(self, step: int) -> None:
        self.step_ctr.fill_(int(step))
        if getattr(self, "_one", None) is not None:
            self._one.reset()  # the published-step flag must not match a rewound step

    def gradients_once(self) -> np.ndarray:
        """Run fwd/bwd on the current batch WITHOUT updating; return the tile-native gradient (index it with
        `self.gidx_np` for canonical order)."""
        self._launch(self.records, self.n_data, self.batch, 0, self.step_ctr, self.slab, self.slab_loss, None,
                     self.grid, True)
        if self.grid > 1:
            wdk.reduce(self.slab, self.grid, 1, self.grad)
            return self.grad[0].cpu().numpy()
        return self.slab[0].cpu().numpy()

    @torch.no_grad()
    def predict_logits(self, records: torch.Tensor) -> torch.Tensor:
        records = records.to(self.device).contiguous()
        n = records.shape[0]
        out = torch.empty(n, device=self.device)
        grid = min((n + self.T - 1) // self.T, 1024)
        self._launch(records, n, n, 0, None, None, None, out, grid, False)
        return out

    def sync_to_model(self) -> wdm.WideDeepModel:
        p = self.param.cpu()
        self._check_exchange()
        return wdm.unpack_canonical(p, self.model)

    def state_dict(self) -> dict:
        return {"param": self.param.cpu(), "s0": self.s0.cpu(), "s1": self.s1.cpu(), "step": self.step_ctr[:1].cpu()}

    def load_state_dict(self, sd: dict) -> None:
        self.set_master_state(sd["param"], sd["s0"], sd["s1"])
        self.set_step(int(sd["step"].reshape(-1)[0]))
