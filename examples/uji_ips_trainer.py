#!/usr/bin/env python3
"""UJIIndoorLoc WiFi positioning MLP (reference examples/uji_ips_trainer.cpp): 520 RSSI features
-> dense 192-64-32-16 (BN + ReLU + dropout) -> (longitude, latitude), trained with the squared
Euclidean *distance in metres* (targets de-normalised inside the loss; gradient chained through
the target std).  Falls back to a synthetic fingerprint set when ./data/uji is absent.
"""
import os

import numpy as np
import torch
from common import parse

from dcnn_amd.data import ArrayDataLoader, WiFiDataLoader
from dcnn_amd.nn import Adam, Loss, SequentialBuilder, TrainingConfig
from dcnn_amd.runtime.step import TrainStep


class DistanceLoss(Loss):
    kind = "distance"

    def __init__(self, target_std):
        super().__init__()
        self.std = torch.as_tensor(np.asarray(target_std[:2], dtype=np.float32))

    def loss_and_grad(self, pred, target, want_grad=True):
        p = pred.reshape(pred.shape[0], -1).float()
        t = target.reshape(p.shape).float()
        s = self.std.to(p.device)
        diff = (p[:, :2] - t[:, :2]) * s            # metres
        loss = (diff * diff).sum(1).mean().view(1)
        grad = None
        if want_grad:
            g = torch.zeros_like(p)
            g[:, :2] = 2.0 / p.shape[0] * diff * s
            grad = g.view(pred.shape).to(pred.dtype)
        return loss, grad, None


def synthetic(n, seed):
    g = np.random.default_rng(seed)
    aps = g.uniform(0, 100, (520, 2))
    pos = g.uniform(0, 100, (n, 2)).astype(np.float32)
    d = np.linalg.norm(pos[:, None, :] - aps[None], axis=2)
    rssi = np.where(d < 40, -30 - 1.5 * d + g.normal(0, 2, d.shape), 100).astype(np.float32)
    return rssi, pos


a, cfg = parse(__doc__)
tr, te = WiFiDataLoader(True), WiFiDataLoader(True)
f_tr, f_te = os.path.join(a.data, "uji", "TrainingData.csv"), os.path.join(a.data, "uji", "ValidationData.csv")
if os.path.exists(f_tr) and not a.synthetic:
    tr.load_data(f_tr, 0, 520, 520, 522)
    te.load_data(f_te, 0, 520, 520, 522)
else:
    print("UJI dataset not found: using synthetic fingerprints")
    for ld, (x, y) in ((tr, synthetic(4000, 1)), (te, synthetic(800, 2))):
        x = np.where((x == 100) | (x == 0), -100, x).astype(np.float32)
        ld.set_arrays(x, y)
tr.normalize_data()
te.normalize_data(stats_from=tr)
model = (SequentialBuilder("uji_ips").input([520, 1, 1]).flatten()
         .dense(192, True, "hidden1").batchnorm(1e-5, 0.1, True, "batchnorm1").activation("relu").dropout(0.25)
         .dense(64, True, "hidden2").batchnorm(1e-5, 0.1, True, "batchnorm2").activation("relu")
         .dense(32, True, "hidden3").batchnorm(1e-5, 0.1, True, "batchnorm3").activation("relu").dropout(0.25)
         .dense(16, True, "hidden4").batchnorm(1e-5, 0.1, True, "batchnorm4").activation("relu")
         .dense(2, True, "output").build())
model.set_device(a.device)
model.initialize()
loss = DistanceLoss(tr.target_std)
opt = Adam(1e-3)
opt.attach(model)
step = TrainStep(model, loss, opt)
dev = model.device.torch_device
tr_ld = ArrayDataLoader(tr.data.reshape(-1, 520, 1, 1), tr.labels, batch_size=cfg.batch_size, shuffle=True)
te_ld = ArrayDataLoader(te.data.reshape(-1, 520, 1, 1), te.labels, batch_size=cfg.batch_size)
for ep in range(cfg.epochs):
    model.set_training(True)
    tot, nb = 0.0, 0
    for x, y in tr_ld:
        tot += float(step(x.to(dev), y.to(dev)))
        nb += 1
        if a.max_batches and nb >= a.max_batches:
            break
    model.set_training(False)
    errs = []
    for x, y in te_ld:
        out = model.forward(x.to(dev), 0, return_on_input_device=False).float().reshape(x.shape[0], -1)
        model.clear_cache(0)
        errs.append(torch.linalg.vector_norm((out[:, :2].cpu() - y[:, :2]) * loss.std, dim=1))
    err = torch.cat(errs)
    print(f"Epoch {ep + 1}/{cfg.epochs}: train distance^2 {tot / max(nb, 1):.2f} m^2 | "
          f"val mean error {err.mean():.2f} m, median {err.median():.2f} m", flush=True)
