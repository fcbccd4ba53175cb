"""ModelOps for arbitrary user PyTorch models (reference:
metisfl/models/pytorch/pytorch_model_ops.py:22-172).

Fixes vs the reference: weights are exported as
``state_dict`` entries in order, parameters marked trainable and buffers
(BN running stats) non-trainable, so set/get round-trip exactly (the
reference zips ``named_parameters`` values onto ``state_dict`` keys); the
model runs on the GPU (the reference's device code is commented out); the
task reports real completed batches and timings (the reference reports 0, so
its batch scaler sees zeros).

Training: all parameters are re-pointed into ONE flat fp32 buffer (and their
gradients into one flat gradient buffer), so the optimizer is a single fused
HIP launch over the whole model (ops/optim.py) instead of one kernel per
tensor.  A TorchModelDef may override ``fit(model, dataset, epochs)`` to keep
full control of the loop, like the reference's PyTorchDef."""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from metisfl_amd.models.model_ops import ModelOps, TaskCancelled
from metisfl_amd.models.model_proto_factory import ModelProtoFactory
from metisfl_amd.ops import optim as opt_ops
from metisfl_amd.ops.optim import OptimizerSpec


class TorchModelOps(ModelOps):

    def __init__(self, model_def, device="cuda", seed: int = 0, he_scheme=None):
        super().__init__(he_scheme)
        torch.manual_seed(seed)
        self.model_def = model_def
        self.device = torch.device(device)
        self.model = model_def.get_model().to(self.device)
        self._flatten()
        self.spec: OptimizerSpec | None = None
        self.m = self.v = self.anchor = None
        self.step = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.lr_scale = torch.ones(1, dtype=torch.float32, device=self.device)

    def _flatten(self):
        params = [p for p in self.model.parameters() if p.requires_grad]
        n = sum(p.numel() for p in params)
        pad = (-n) % 4
        self.flat = torch.zeros(n + pad, dtype=torch.float32, device=self.device)
        self.flat_grad = torch.zeros_like(self.flat)
        off = 0
        for p in params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1).float())
            p.data = self.flat[off:off + k].view_as(p)
            p.grad = self.flat_grad[off:off + k].view_as(p)
            off += k
        self.params = params

    # -- weights -----------------------------------------------------------------------
    def get_model_weights(self):
        sd = self.model.state_dict()
        pnames = {n for n, _ in self.model.named_parameters()}
        names = list(sd.keys())
        return names, [n in pnames for n in names], [sd[n].detach().cpu().numpy().copy() for n in names]

    def set_model_weights(self, names, arrays):
        sd = self.model.state_dict()
        if set(names) != set(sd.keys()):
            if len(names) != len(sd):
                raise ValueError(f"model has {len(names)} variables, expected {len(sd)}")
            names = list(sd.keys())  # positional
        with torch.no_grad():
            for n, a in zip(names, arrays):
                sd[n].copy_(torch.as_tensor(np.asarray(a)).reshape(sd[n].shape).to(sd[n].dtype))
        if self.anchor is not None:
            self.anchor.copy_(self.flat)

    # -- optimizer -----------------------------------------------------------------------
    def construct_optimizer(self, optimizer_config_pb):
        spec = OptimizerSpec.from_proto(optimizer_config_pb)
        if self.spec is None or spec.kind != self.spec.kind:
            self.m = torch.zeros_like(self.flat) if spec.needs_m else None
            self.v = torch.zeros_like(self.flat) if spec.needs_v else None
            self.anchor = self.flat.clone() if spec.needs_anchor else None
        self.spec = spec

    def _batches(self, ds, batch_size, shuffle, gen):
        x = torch.as_tensor(np.asarray(ds.get_x())).float()
        y = torch.as_tensor(np.asarray(ds.get_y()))
        n = x.shape[0]
        idx = torch.randperm(n, generator=gen) if shuffle else torch.arange(n)
        for i in range(0, n, batch_size):
            j = idx[i:i + batch_size]
            yield x[j].to(self.device, non_blocking=True), y[j].to(self.device, non_blocking=True)

    def train_model(self, train_dataset, learning_task_pb, hyperparameters_pb, validation_dataset=None,
                    test_dataset=None, verbose=False, cancel_event=None):
        B = int(hyperparameters_pb.batch_size) or 32
        if hyperparameters_pb.HasField("optimizer"):
            self.construct_optimizer(hyperparameters_pb.optimizer)
        elif self.spec is None:
            self.spec = OptimizerSpec()
        total = int(learning_task_pb.num_local_updates)
        spe = max(1, math.ceil(train_dataset.get_size() / B))
        gen = torch.Generator().manual_seed(int(learning_task_pb.global_iteration))
        self.model.train()
        stats = {"loss": [], "accuracy": []}
        done = 0
        t0 = time.perf_counter()
        user_fit = getattr(self.model_def, "fit", None)
        if callable(user_fit):
            user_fit(self.model, train_dataset, max(1, math.ceil(total / spe)))
            done = total
        else:
            while done < total:
                tot_loss = tot_acc = cnt = 0.0
                for xb, yb in self._batches(train_dataset, B, True, gen):
                    if cancel_event is not None and cancel_event.is_set():
                        raise TaskCancelled()
                    out = self.model(xb)
                    loss = self.model_def.loss(out, yb)
                    loss.backward()
                    opt_ops.fused_step(self.spec, self.flat, self.flat_grad, self.m, self.v, self.anchor, None,
                                       self.lr_scale, self.step, zero_grad=True)
                    opt_ops.tick(self.step, 1)
                    tot_loss += float(loss.detach()) * xb.shape[0]
                    if out.dim() == 2 and out.shape[1] > 1:
                        tot_acc += float((out.argmax(1) == yb).sum())
                    cnt += xb.shape[0]
                    done += 1
                    if done >= total:
                        break
                stats["loss"].append(tot_loss / max(1, cnt))
                stats["accuracy"].append(tot_acc / max(1, cnt))
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        ms = (time.perf_counter() - t0) * 1e3
        val = self.evaluate_model(validation_dataset, B) if validation_dataset is not None and \
            validation_dataset.get_size() else {}
        test = self.evaluate_model(test_dataset, B) if test_dataset is not None and test_dataset.get_size() else {}
        names, trainable, values = self.get_model_weights()
        msg = ModelProtoFactory.CompletedLearningTaskProtoMessage(
            names, trainable, values, stats, done / spe, learning_task_pb.global_iteration, val, test, done, B,
            ms / max(1, done) * spe, ms / max(1, done))
        return msg.construct_completed_learning_task_pb(he_scheme=self.he_scheme)

    @torch.no_grad()
    def evaluate_model(self, dataset, batch_size, metrics=(), verbose=False, model_pb=None) -> dict:
        if dataset is None or not dataset.get_size():
            return {}
        model = self.model
        if model_pb is not None:  # community model: separate copy, training may be running
            import copy
            if getattr(self, "eval_model", None) is None:
                self.eval_model = copy.deepcopy(self.model)
            model = self.eval_model
            names, arrays = self.get_model_weights_from_variables_pb(model_pb)
            sd = model.state_dict()
            keys = names if set(names) == set(sd) else list(sd)
            for n, a in zip(keys, arrays):
                sd[n].copy_(torch.as_tensor(np.asarray(a)).reshape(sd[n].shape).to(sd[n].dtype))
        user_eval = getattr(self.model_def, "evaluate", None)
        if callable(user_eval):
            res = dict(user_eval(model, dataset))
        else:
            model.eval()
            tot_loss = tot_acc = cnt = 0.0
            for xb, yb in self._batches(dataset, int(batch_size) or 32, False, None):
                out = model(xb)
                tot_loss += float(self.model_def.loss(out, yb)) * xb.shape[0]
                if out.dim() == 2 and out.shape[1] > 1:
                    tot_acc += float((out.argmax(1) == yb).sum())
                cnt += xb.shape[0]
            model.train()
            res = {"loss": tot_loss / max(1, cnt), "accuracy": tot_acc / max(1, cnt)}
        return res
